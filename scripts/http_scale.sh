# CPU share probe + HTTP hit-path scaling with proxy / load-generator threads
set -o pipefail
mkdir -p gpurun_out
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/self/status | grep -i cpus_allowed_list; grep -m1 "model name" /proc/cpuinfo; } > gpurun_out/cpu_probe.txt 2>&1
for cfg in "8 8" "12 8" "16 12"; do
  set -- $cfg
  timeout -k 10 250 python benchmarks/http_bench.py --backend tiered --objects 1000000 --requests 2000000 --conc 1000 --threads $1 --client-threads $2 --out gpurun_out/http_tiered_t$1_c$2.json > gpurun_out/http_tiered_t$1_c$2.log 2>&1 || { tail -5 gpurun_out/http_tiered_t$1_c$2.log; exit 1; }
  echo "threads $1 client $2: $(grep 'c=1000' gpurun_out/http_tiered_t$1_c$2.log)"
done
cat gpurun_out/cpu_probe.txt
