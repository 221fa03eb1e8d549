#!/bin/bash
# The routed serving step on one GPU: routed GPU tests, then the simulated 8- and 2-rank
# steps, the one-rank RCCL step and the N=1 headline (each with --check), each under its
# own limit. `bash scripts/routed_check.sh OUT [extra bench args]`; output in gpurun_out/OUT.
set -o pipefail
OUT=gpurun_out/${1:-routed_check}
shift || true
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_hbm_gpu.py -k "routed or overflow or serve_get_multi" tests/test_routed_multiproc_gpu.py \
  tests/test_index_relocation.py \
  > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
for args in "--simulate-world 8" "--simulate-world 2" "--routed" ""; do
  name=$(echo "x$args" | tr -d ' -')
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --check --no-uncoalesced \
    --no-wrapped "$@" $args > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" \
    || { echo "bench $args failed"; tail -30 "$OUT/bench_$name.err"; exit 1; }
  echo "== $args"; grep check "$OUT/bench_$name.err"; cut -c1-300 "$OUT/bench_$name.json"
done
