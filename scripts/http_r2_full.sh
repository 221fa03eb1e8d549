# Round-2 HTTP matrix: {dram L1-size only, tiered HBM+L1} x {1K, 1M, 8M objects of 4 KiB,
# 256K objects of 64 KiB}; origin and load generator in their own processes
set -o pipefail
mkdir -p gpurun_out/http
run() { # name args...
  local name=$1; shift
  timeout -k 10 400 python benchmarks/http_bench.py "$@" --out gpurun_out/http/$name.json > gpurun_out/http/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/http/$name.log; return 1; }
  grep "\[http\]" gpurun_out/http/$name.log | sed "s|^|$name |" | cut -c1-220
}
run dram_1K   --backend dram   --objects 1000    --requests 1000000 && \
run tiered_1K --backend tiered --objects 1000    --requests 1000000 && \
run dram_8M   --backend dram   --objects 8000000 --requests 1000000 --timeout 600 && \
run tiered_8M --backend tiered --objects 8000000 --requests 1000000 --timeout 600 && \
run dram_256K_64k   --backend dram   --objects 262144 --body 65536 --requests 200000 && \
run tiered_256K_64k --backend tiered --objects 262144 --body 65536 --requests 200000
