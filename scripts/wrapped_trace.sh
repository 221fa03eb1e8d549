#!/usr/bin/env bash
# Kernel trace of the N=1 step with the value log wrapped (steady state: the CLOCK hand
# runs before every SET batch), at the default 16 GiB log and at 5 GiB.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for cfg in "16:400" "5:80"; do
  lg=${cfg%%:*}; wu=${cfg#*:}
  OUT=gpurun_out/wt_trace
  timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $OUT -o bench -- \
    python3 bench.py --log-gb $lg --warmup $wu --steps 10 --no-smoke --no-uncoalesced --no-wrapped > /dev/null 2>&1 \
    && python scripts/step_kernel_stats.py $(ls $OUT/bench_kernel_trace.csv $OUT/*/bench_kernel_trace.csv 2>/dev/null | head -1) \
       --title "N=1 step, $lg GiB log wrapped (CLOCK)" > gpurun_out/wrapped_${lg}g_kernel_stats.md
  rm -rf $OUT
done
