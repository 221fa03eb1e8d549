#!/bin/bash
# The driver's round-end tiers on one GPU: the whole GPU suite, smoke(), the N=1 bench.
set -o pipefail
OUT=gpurun_out/${1:-r3_final}
mkdir -p "$OUT"
bash scripts/r3_gpu_suite.sh "${1:-r3_final}" && \
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" && \
  bash scripts/r3_bench_default.sh "${1:-r3_final}"
