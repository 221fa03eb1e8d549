#!/bin/bash
# HTTP matrix (8M x 4 KiB incompressible, Zipf 0.99, c=10 and c=1000): DRAM-only,
# HBM-only and tiered, the GPU batcher on a core of its own (8 reactors x 6 load-generator
# workers), HBM-only also without reactor-direct jobs (every GET through the batcher thread),
# with 1 or 4 edge-server blocks instead of 8 (hbm_blk1, hbm_blk4)
# and without the resident edge server (a launch per GET batch); hbm2 / hbm2_nohot: two HBM
# shards on GPU 0 (a stand-in for two GPUs) with and without hot-object spreading.
set -o pipefail
OUT=gpurun_out/${1:-http_matrix}
mkdir -p "$OUT"
run() { # name args...
  local name=$1; shift
  timeout -k 10 560 python benchmarks/http_bench.py "$@" --out "$OUT/$name.json" \
    > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; return 1; }
  grep "\[http\]" "$OUT/$name.log" | sed "s|^|$name |" | cut -c1-260
}
shift
for spec in "$@"; do
  case $spec in
    dram)   run dram_8M   --backend dram   --objects 8000000 --requests 2000000 --conc 10 1000 --layouts 8x6 --timeout 400 || exit 1;;
    hbm)    run hbm_8M    --backend hbm    --objects 8000000 --requests 2000000 --conc 10 1000 --layouts 8x6 --timeout 400 || exit 1;;
    hbm_b1) run hbm_8M_backlog1 --backend hbm --objects 8000000 --requests 2000000 --conc 10 1000 --layouts 8x6 --timeout 400 --serve-backlog 1 || exit 1;;
    hbm_blk1) run hbm_8M_blk1 --backend hbm --objects 8000000 --requests 2000000 --conc 10 1000 --layouts 8x6 --timeout 400 --serve-blocks 1 || exit 1;;
    hbm_blk4) run hbm_8M_blk4 --backend hbm --objects 8000000 --requests 2000000 --conc 10 1000 --layouts 8x6 --timeout 400 --serve-blocks 4 || exit 1;;
    hbm_nodirect) run hbm_8M_nodirect --backend hbm --objects 8000000 --requests 2000000 --conc 10 1000 --layouts 8x6 --timeout 400 --no-direct || exit 1;;
    hbm_nosrv) run hbm_8M_nosrv --backend hbm --objects 8000000 --requests 2000000 --conc 10 1000 --layouts 8x6 --timeout 400 --no-edge-server || exit 1;;
    hbm2)   run hbm2_8M   --backend hbm    --objects 8000000 --requests 2000000 --conc 10 1000 --layouts 7x6 --timeout 400 --shards 2 || exit 1;;
    hbm2_nohot) run hbm2_8M_nohot --backend hbm --objects 8000000 --requests 2000000 --conc 10 1000 --layouts 7x6 --timeout 400 --shards 2 --hot-objects 0 || exit 1;;
    tiered) run tiered_8M --backend tiered --objects 8000000 --requests 2000000 --conc 10 1000 --layouts 8x6 --timeout 400 || exit 1;;
  esac
done
