#!/bin/bash
# Timeline of the round-6 headline step (walk stream, working set = log): kernel trace of the
# default bench minus the cycled / overfull blocks, so the last steps are the headline
# block's; summarised on the box.
set -o pipefail
OUT=${1:-r6_trace}
mkdir -p gpurun_out/$OUT
TRACE_OUT=$OUT/raw TRACE_LIMIT=300 bash scripts/trace_bench.sh --no-uncoalesced --no-cycled \
  --overfull-fill 0 > gpurun_out/$OUT/trace.log 2>&1 || { tail -20 gpurun_out/$OUT/trace.log; exit 1; }
python3 scripts/step_trace_summary.py gpurun_out/$OUT/raw 8 hbm.lookup_coalesced > gpurun_out/$OUT/pressured_walk_summary.txt
STEP_TABLE=1 SPAN=4 python3 scripts/step_trace_summary.py gpurun_out/$OUT/raw 40 hbm.lookup_coalesced > gpurun_out/$OUT/pressured_walk_steps.txt
rm -rf gpurun_out/$OUT/raw
head -40 gpurun_out/$OUT/pressured_walk_summary.txt
