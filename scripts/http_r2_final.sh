# Round-2 HTTP matrix with the final bench defaults: 9 reactors + 6 load-generator
# workers on their own cores of socket 0 (busy-polling 200 us), the GPU batcher, the
# proxy's other threads and the origin on a 16th core (the box's cgroup quota is 16 CPUs).
# Objects: 4 KiB incompressible bodies, 1K / 8M objects; 64 KiB bodies, 256K objects.
set -o pipefail
mkdir -p gpurun_out/http_final
run() { # name args...
  local name=$1; shift
  timeout -k 10 500 python benchmarks/http_bench.py "$@" --out gpurun_out/http_final/$name.json \
    > gpurun_out/http_final/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/http_final/$name.log; return 1; }
  grep "\[http\]" gpurun_out/http_final/$name.log | sed "s|^|$name |" | cut -c1-250
}
run dram_1K     --backend dram   --objects 1000    --requests 1000000 && \
run tiered_1K   --backend tiered --objects 1000    --requests 1000000 && \
run dram_8M     --backend dram   --objects 8000000 --requests 2000000 --timeout 400 && \
run tiered_8M   --backend tiered --objects 8000000 --requests 2000000 --timeout 400 && \
run hbm_8M      --backend hbm    --objects 8000000 --requests 2000000 --timeout 400 && \
run dram_256K_64k   --backend dram   --objects 262144 --body 65536 --requests 300000 && \
run tiered_256K_64k --backend tiered --objects 262144 --body 65536 --requests 300000
