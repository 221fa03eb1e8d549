#!/bin/bash
# The round-end checks on one box, in the driver's order, for the record: the GPU suite
# (scripts/gpu_tests.sh), smoke(), the driver's N=1 bench command, and a kernel-trace
# summary of a short bench run (rocprofv3 --kernel-trace --stats). Output gpurun_out/OUT.
set -o pipefail
OUT=${1:-r6_final_check}
mkdir -p gpurun_out/$OUT
bash scripts/gpu_tests.sh $OUT/tests || exit 1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$OUT/smoke.log 2>&1 \
  || { tail -20 gpurun_out/$OUT/smoke.log; exit 1; }
tail -1 gpurun_out/$OUT/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/$OUT/bench.json 2> gpurun_out/$OUT/bench.err \
  || { tail -30 gpurun_out/$OUT/bench.err; exit 1; }
cut -c1-600 gpurun_out/$OUT/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$OUT/prof -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-smoke --no-uncoalesced > gpurun_out/$OUT/prof.log 2>&1 \
  || { tail -20 gpurun_out/$OUT/prof.log; exit 1; }
f=$(find gpurun_out/$OUT/prof -name "*kernel_stats.csv" | head -1)
head -25 "$f" | cut -c1-200 > gpurun_out/$OUT/kernel_stats_top.csv
find gpurun_out/$OUT/prof -name "*kernel_trace.csv" -delete
cat gpurun_out/$OUT/kernel_stats_top.csv | cut -d, -f1-6 | head -16
