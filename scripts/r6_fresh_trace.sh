#!/bin/bash
# Timeline of the pre-wrap step (log_fresh: no CLOCK hand, nothing overwritten): kernel trace
# of the bench with only the fresh phase, summarised on the box with the GPU-clock span of
# the last 4 steps.
set -o pipefail
OUT=${1:-r6_fresh_trace}
mkdir -p gpurun_out/$OUT
TRACE_OUT=$OUT/raw TRACE_LIMIT=300 bash scripts/trace_bench.sh --no-uncoalesced --no-wrapped \
  --pressured-gb 0 --headline fresh > gpurun_out/$OUT/trace.log 2>&1 || { tail -20 gpurun_out/$OUT/trace.log; exit 1; }
STEP_TABLE=1 SPAN=4 python3 scripts/step_trace_summary.py gpurun_out/$OUT/raw 8 hbm.lookup_coalesced > gpurun_out/$OUT/fresh_steps.txt
rm -rf gpurun_out/$OUT/raw
sed -n '/last 4 steps/,$p' gpurun_out/$OUT/fresh_steps.txt | head -60
