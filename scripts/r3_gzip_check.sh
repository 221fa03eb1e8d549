#!/bin/bash
# Round 3: GPU gzip after the device-side planning + lane-parallel lazy parse:
# zlib-verified tests, the batch throughput/ratio bench, the proxy's -z miss path.
set -o pipefail
OUT=gpurun_out/${1:-r3_gzip}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_gzip.py > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 300 python -u benchmarks/gzip_bench.py --sizes 8192 65536 --count 2048 --reps 3 \
  > "$OUT/gzip_bench.log" 2>&1 || { echo "gzip bench failed"; tail -30 "$OUT/gzip_bench.log"; exit 1; }
cat "$OUT/gzip_bench.log" | tail -12
if [ "${2:-}" = "http" ]; then
  timeout -k 10 500 python -u benchmarks/http_compress_bench.py --objects 100000 --modes cpu gpu \
    > "$OUT/http_compress.jsonl" 2> "$OUT/http_compress.err" || { echo "http bench failed"; tail -30 "$OUT/http_compress.err"; exit 1; }
  cut -c1-400 "$OUT/http_compress.jsonl"
fi
