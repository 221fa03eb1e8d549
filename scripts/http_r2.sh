set -o pipefail
mkdir -p gpurun_out
for b in dram tiered hbm; do
  timeout -k 10 280 python benchmarks/http_bench.py --backend $b --objects 1000000 --requests 1000000 --conc 10 1000 --threads 8 --client-threads 4 --out gpurun_out/http_${b}_1M.json > gpurun_out/http_${b}_1M.log 2>&1 || { echo "$b failed"; tail -20 gpurun_out/http_${b}_1M.log; exit 1; }
  grep "\[http\]" gpurun_out/http_${b}_1M.log
done
