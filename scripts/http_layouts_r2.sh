# Layout sweep after the arena/fd-table fixes: tiered 8M x 4 KiB at c=1000, one filled
# cache (the first layout also warms the L1 after the fill; 9x5 and 9x6 measured twice),
# cache, a proxy per RxC layout (core 14 is free under the default 9x5)
set -o pipefail
mkdir -p gpurun_out/http_lay
timeout -k 10 900 python benchmarks/http_bench.py --backend tiered --objects 8000000 \
  --requests 2000000 --conc 1000 --timeout 600 --layouts 9x5 9x6 10x5 9x5 9x6 \
  --out gpurun_out/http_lay/tiered_8M_layouts.json > gpurun_out/http_lay/tiered_8M_layouts.log 2>&1
rc=$?; grep "\[http\]" gpurun_out/http_lay/tiered_8M_layouts.log | cut -c1-230; exit $rc
