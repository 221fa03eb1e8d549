# Connection-setup diagnosis: per-core user/system/irq/softirq/idle around each run
set -o pipefail
mkdir -p gpurun_out/http_diag
name=I_1000_10_1000
timeout -k 10 300 python benchmarks/http_bench.py --objects 2000000 --requests 1000000 --timeout 200 \
  --backend hbm --conc 1000 10 1000 --out gpurun_out/http_diag/$name.json > gpurun_out/http_diag/$name.log 2>&1
rc=$?
grep -c . /proc/interrupts > /dev/null
grep -i "amdgpu\|kfd" /proc/interrupts | cut -c1-200 | head -5 > gpurun_out/http_diag/irq.txt || true
cat /proc/irq/*/smp_affinity_list > /dev/null 2>&1 || true
exit $rc
