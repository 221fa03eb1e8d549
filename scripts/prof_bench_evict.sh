# rocprofv3 kernel stats of the N=1 bench step under CLOCK and FIFO eviction
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out
for ev in clock fifo; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --evict $ev --no-uncoalesced --no-smoke > gpurun_out/bench_$ev.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$ev -o run -- python3 bench.py --steps 20 --warmup 5 --evict $ev --no-uncoalesced --no-smoke > gpurun_out/prof_$ev.log 2>&1 || exit 1
done
grep -h ms_per_step gpurun_out/bench_clock.log gpurun_out/bench_fifo.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['config']['model'], d['ms_per_step'], d.get('ms_per_step_median_gpu_events'))"
find gpurun_out/prof_clock gpurun_out/prof_fifo -name "*kernel_stats.csv" | head
