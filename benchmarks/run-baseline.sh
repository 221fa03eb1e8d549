#!/usr/bin/env bash
# Origin alone (reference: benchmarks/run-baseline.sh, `ab ... http://127.0.0.1/`).
# usage: run-baseline.sh [origin_port]
cd "$(dirname "$0")/.."
python3 -m shellac_amd.bench.ab -k -n 400 -c 10 -g benchmarks/baseline.dat -H "Accept-Encoding: gzip" "http://127.0.0.1:${1:-80}/"
