#!/bin/bash
# The driver's N=1 headline run (bench.py defaults: log_wrapped + log_pressured blocks).
set -o pipefail
OUT=gpurun_out/${1:-bench_default}
mkdir -p "$OUT"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cut -c1-3000 "$OUT/bench.json"
