# Reactor busy-poll A/B (proxy --spin-us) on the tiered 8M-object workload, c=1000;
# a fresh process per configuration
set -o pipefail
mkdir -p gpurun_out/http_pin
run() { # name args...
  local name=$1; shift
  timeout -k 10 500 python benchmarks/http_bench.py --backend tiered --objects 8000000 \
    --requests 2000000 --conc 1000 --timeout 400 "$@" --out gpurun_out/http_pin/$name.json \
    > gpurun_out/http_pin/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/http_pin/$name.log; return 1; }
  grep "\[http\]" gpurun_out/http_pin/$name.log | sed "s|^|$name |" | cut -c1-260
}
run t8M_9x5_spin200b --layouts 9x5 --rx-spin-us 200 && \
run t8M_8x6_spin200 --layouts 8x6 --rx-spin-us 200 && \
run t8M_8x6_spin0 --layouts 8x6 --rx-spin-us 0
