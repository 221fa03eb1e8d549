# Thread-layout sweep on the 16-CPU box: one filled cache (tiered, 8M objects of 4 KiB),
# a proxy per RxC layout (R reactors, C load-generator workers, each on its own core;
# the GPU batcher, the proxy's other threads and the origin share the last core)
set -o pipefail
mkdir -p gpurun_out/http_pin
timeout -k 10 900 python benchmarks/http_bench.py --backend tiered --objects 8000000 \
  --requests 2000000 --conc 1000 --timeout 600 --misc-cpus 1 --layouts 9x5 10x5 11x4 9x6 10x4 \
  --out gpurun_out/http_pin/tiered_8M_layouts2.json > gpurun_out/http_pin/tiered_8M_layouts2.log 2>&1
rc=$?; grep "\[http\]" gpurun_out/http_pin/tiered_8M_layouts2.log | cut -c1-260; exit $rc
