#!/bin/bash
# N=1 iteration: the serve-path GPU tests, the default bench twice, a kernel trace summary.
set -o pipefail
OUT=gpurun_out/${1:-r3_n1}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_hbm_gpu.py tests/test_bench_contract.py -m gpu > "$OUT/tests.log" 2>&1 \
  || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --check --no-smoke > "$OUT/bench$i.json" 2> "$OUT/bench$i.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench$i.err"; exit 1; }
  grep check "$OUT/bench$i.err"; cut -c1-200 "$OUT/bench$i.json"
  python3 -c "import json;d=json.load(open('$OUT/bench$i.json'));print('wrapped',d['log_wrapped']['ms_per_step'],'pressured',d['log_pressured']['ms_per_step'],'unco',d['uncoalesced_ops_per_s'])"
done
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT/trace" -o bench -- \
  python3 "$R/bench.py" --steps 10 --warmup 3 --no-smoke --no-uncoalesced --no-wrapped --pressured-gb 0 \
  > "$R/$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -20 "$R/$OUT/trace.log"; exit 1; }
f=$(find "$R/$OUT/trace" -name '*kernel_trace.csv' | head -1)
python3 "$R/scripts/step_kernel_stats.py" "$f" --steps 8 --title "N=1 pipelined lookup" > "$R/$OUT/kernel_stats.md"
head -40 "$R/$OUT/kernel_stats.md"
rm -rf "$R/$OUT/trace"
