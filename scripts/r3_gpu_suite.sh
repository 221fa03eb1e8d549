#!/bin/bash
# The driver's round-end GPU tier: the whole `pytest -m gpu` suite in one process.
set -o pipefail
OUT=gpurun_out/${1:-r3_suite}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  > "$OUT/gpu_suite.log" 2>&1 || { echo "gpu suite failed"; tail -60 "$OUT/gpu_suite.log"; exit 1; }
tail -3 "$OUT/gpu_suite.log"
