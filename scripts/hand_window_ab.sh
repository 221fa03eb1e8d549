#!/usr/bin/env bash
# Steady-state (log wrapped) N=1 step vs the CLOCK hand's window (SHELLAC_HAND_WINDOW=k:
# k*n + 256 ring entries per SET batch of n rows), at the default 16 GiB log and at 5 GiB;
# plus a kernel trace of the 16 GiB steady state at the default k.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
run() {
  timeout -k 10 150 python bench.py --steps 20 --no-smoke --no-uncoalesced --check "$@" 2> gpurun_out/hw_err.log \
    | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print("ms/step", j["ms_per_step"], "median", j.get("ms_per_step_median_gpu_events"), "hit", j["get_hit_ratio"], "reinsert MB/step %.1f" % (j["reinserted_bytes_per_step"] / 1e6))' \
    || { tail -5 gpurun_out/hw_err.log; exit 1; }
  grep -h "check:" gpurun_out/hw_err.log | tr '\n' ' '; echo
}
for k in 4 2 1; do
  echo "== k=$k log 16 GiB warmup 400"; SHELLAC_HAND_WINDOW=$k run --warmup 400
  echo "== k=$k log 5 GiB warmup 80"; SHELLAC_HAND_WINDOW=$k run --log-gb 5 --warmup 80
done
OUT=gpurun_out/hw_trace
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $OUT -o bench -- \
  python3 bench.py --warmup 400 --steps 10 --no-smoke --no-uncoalesced > /dev/null 2>&1 \
  && python scripts/step_kernel_stats.py $(ls $OUT/bench_kernel_trace.csv $OUT/*/bench_kernel_trace.csv 2>/dev/null | head -1) \
     --title "N=1 step, 16 GiB log in steady state (CLOCK, window 4n)" > gpurun_out/hw_kernel_stats_16g.md
rm -rf $OUT
