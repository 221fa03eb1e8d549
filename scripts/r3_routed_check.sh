#!/bin/bash
# Round 3: the device-driven routed step on one GPU — routed GPU tests, the simulated
# 8-rank step, the one-rank RCCL step and the N=1 headline, each under its own limit.
set -o pipefail
OUT=gpurun_out/${1:-r3_routed}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_hbm_gpu.py -k "routed or overflow" tests/test_routed_multiproc_gpu.py \
  > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
for args in "--simulate-world 8" "--simulate-world 2" "--routed" ""; do
  name=$(echo "x$args" | tr -d ' -')
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --check --no-uncoalesced \
    --no-wrapped $args > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" \
    || { echo "bench $args failed"; tail -30 "$OUT/bench_$name.err"; exit 1; }
  echo "== $args"; grep check "$OUT/bench_$name.err"; cut -c1-300 "$OUT/bench_$name.json"
done
