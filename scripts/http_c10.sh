# c=10 vs c=1000 with busy-polling reactors and load-generator workers on pinned cores
set -o pipefail
mkdir -p gpurun_out/http_pin
run() { # name args...
  local name=$1; shift
  timeout -k 10 500 python benchmarks/http_bench.py "$@" --out gpurun_out/http_pin/$name.json \
    > gpurun_out/http_pin/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/http_pin/$name.log; return 1; }
  grep "\[http\]" gpurun_out/http_pin/$name.log | sed "s|^|$name |" | cut -c1-260
}
run t1K_nopin     --backend tiered --objects 1000 --requests 1000000 --conc 10 1000 --pin off && \
run t1K_pin_spin  --backend tiered --objects 1000 --requests 1000000 --conc 10 1000 --rx-spin-us 200 --lg-spin-us 200 && \
run t8M_pin_spin  --backend tiered --objects 8000000 --requests 2000000 --conc 10 1000 --timeout 400 --rx-spin-us 200 --lg-spin-us 200
