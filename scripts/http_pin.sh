# Pinned vs unpinned HTTP runs (benchmarks/http_bench.py --pin auto|off): reactors, load
# generator workers, origin and the GPU batcher each on their own cores of socket 0
set -o pipefail
mkdir -p gpurun_out/http_pin
run() { # name args...
  local name=$1; shift
  timeout -k 10 400 python benchmarks/http_bench.py "$@" --out gpurun_out/http_pin/$name.json > gpurun_out/http_pin/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/http_pin/$name.log; return 1; }
  grep "\[http\]" gpurun_out/http_pin/$name.log | sed "s|^|$name |" | cut -c1-260
}
run tiered_1K_pin   --backend tiered --objects 1000 --requests 1000000 --pin auto && \
run tiered_1K_nopin --backend tiered --objects 1000 --requests 1000000 --pin off && \
run tiered_8M_pin   --backend tiered --objects 8000000 --requests 2000000 --conc 1000 --timeout 600 --pin auto && \
run dram_8M_pin     --backend dram   --objects 8000000 --requests 2000000 --conc 1000 --timeout 600 --pin auto
