#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3_pmc_tests
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_eviction.py -m gpu > gpurun_out/r3_pmc_tests/eviction.log 2>&1 \
  || { echo "eviction tests failed"; tail -30 gpurun_out/r3_pmc_tests/eviction.log; exit 1; }
tail -2 gpurun_out/r3_pmc_tests/eviction.log
bash scripts/r3_pmc.sh
