# The GPU-tier rows of scripts/http_r2_final.sh (after the arena-pool fix)
set -o pipefail
mkdir -p gpurun_out/http_final
run() { # name args...
  local name=$1; shift
  timeout -k 10 500 python benchmarks/http_bench.py "$@" --out gpurun_out/http_final/$name.json \
    > gpurun_out/http_final/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/http_final/$name.log; return 1; }
  grep "\[http\]" gpurun_out/http_final/$name.log | sed "s|^|$name |" | cut -c1-250
}
run tiered_8M   --backend tiered --objects 8000000 --requests 2000000 --timeout 400 && \
run hbm_8M      --backend hbm    --objects 8000000 --requests 2000000 --timeout 400 && \
run tiered_256K_64k --backend tiered --objects 262144 --body 65536 --requests 300000
