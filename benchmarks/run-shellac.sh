#!/usr/bin/env bash
# Through the proxy (reference: benchmarks/run-shellac.sh, port 8080).
cd "$(dirname "$0")/.."
python3 -m shellac_amd.bench.ab -k -n 400 -c 10 -g benchmarks/shellac.dat -H "Accept-Encoding: gzip" "http://127.0.0.1:${1:-8080}/"
