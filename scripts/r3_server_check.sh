#!/bin/bash
# Round 3: the persistent edge-GET server — its GPU tests, the host-observed latency of
# one micro-batch (launch vs resident server), then the HBM backend / proxy GPU tests.
set -o pipefail
OUT=gpurun_out/${1:-r3_server}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_hbm_gpu.py -k "serve_get or small_get or small_set or duplicate or bucket_overflow or roundtrip or fifo or ttl" > "$OUT/server_tests.log" 2>&1 \
  || { echo "server tests failed"; tail -40 "$OUT/server_tests.log"; exit 1; }
tail -2 "$OUT/server_tests.log"
timeout -k 10 300 python -u scripts/small_get_latency.py > "$OUT/edge_get_latency.log" 2>&1 \
  || { echo "latency failed"; tail -30 "$OUT/edge_get_latency.log"; exit 1; }
cat "$OUT/edge_get_latency.log"
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_hbm_backend_gpu.py tests/test_eviction.py -m gpu > "$OUT/backend_tests.log" 2>&1 \
  || { echo "backend tests failed"; tail -40 "$OUT/backend_tests.log"; exit 1; }
tail -2 "$OUT/backend_tests.log"
