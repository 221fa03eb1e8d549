#!/usr/bin/env bash
# Any other accelerator on :6081 (reference: benchmarks/run-varnish.sh).
cd "$(dirname "$0")/.."
python3 -m shellac_amd.bench.ab -k -n 400 -c 10 -g benchmarks/varnish.dat -H "Accept-Encoding: gzip" "http://127.0.0.1:${1:-6081}/"
