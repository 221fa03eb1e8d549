#!/usr/bin/env bash
# The N=1 serving step in steady state under eviction: enough warmup steps that the
# value log has wrapped (so every SET batch runs the CLOCK hand / FIFO overwrite),
# at the default 16 GiB log (4.2 GB live: ~26 % utilisation) and at a 5 GiB log
# (~78 %). Plus a kernel trace of the 5 GiB CLOCK step.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
run() {
  timeout -k 10 150 python bench.py --steps 20 --no-smoke --check "$@" 2> gpurun_out/es_err.log \
    | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print("ms/step", j["ms_per_step"], "median", j.get("ms_per_step_median_gpu_events"), "hit", j["get_hit_ratio"], "unco_ops/s %.3g" % j["uncoalesced_ops_per_s"])' \
    || { tail -5 gpurun_out/es_err.log; exit 1; }
  grep -h "check:" gpurun_out/es_err.log | tr '\n' ' '; echo
}
for w in 5 400; do
  for ev in clock fifo; do
    echo "== log 16 GiB, warmup $w, $ev"; run --warmup $w --evict $ev
  done
done
for ev in clock fifo; do
  echo "== log 5 GiB, warmup 80, $ev"; run --log-gb 5 --warmup 80 --evict $ev
done
OUT=gpurun_out/es_trace
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o bench -- \
  python3 bench.py --log-gb 5 --warmup 80 --steps 10 --no-smoke --no-uncoalesced > /dev/null 2>&1 \
  && python scripts/step_kernel_stats.py $(ls $OUT/bench_kernel_trace.csv $OUT/*/bench_kernel_trace.csv 2>/dev/null | head -1) \
     --title "N=1 step, 5 GiB log in steady state (CLOCK)" > gpurun_out/es_kernel_stats.md
rm -rf $OUT
