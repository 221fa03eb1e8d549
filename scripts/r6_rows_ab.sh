#!/bin/bash
# Round-6 probe: the row-wise gather (one wave per record; SHELLAC_GATHER_ROWS=1 through VGPRs,
# =2 by LDS-DMA) vs k_segcopy<4> (default): the HBM cache's GPU tests with each, then the
# bench alternating on one box, --check on.
set -o pipefail
SHELLAC_GATHER_ROWS=1 bash scripts/gpu_tests.sh r6_rows_ab/tests1 tests/test_hbm_gpu.py -m gpu || exit 1
SHELLAC_GATHER_ROWS=2 bash scripts/gpu_tests.sh r6_rows_ab/tests2 tests/test_hbm_gpu.py -m gpu || exit 1
EXTRA="--no-cycled --overfull-fill 0" bash scripts/env_ab.sh r6_rows_ab \
  "X=1" "SHELLAC_GATHER_ROWS=1" "SHELLAC_GATHER_ROWS=2" "X=1" "SHELLAC_GATHER_ROWS=1" "SHELLAC_GATHER_ROWS=2"
