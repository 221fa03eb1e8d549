#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3_multiproc
SHELLAC_TEST_STACKS=gpurun_out/r3_multiproc timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_routed_multiproc_gpu.py -k "multiprocess" \
  > gpurun_out/r3_multiproc/tests.log 2>&1 || { echo "failed"; tail -40 gpurun_out/r3_multiproc/tests.log; exit 1; }
tail -3 gpurun_out/r3_multiproc/tests.log
