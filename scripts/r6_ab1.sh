#!/bin/bash
# Round-6 batch: the new GPU tests (and the CLOCK twin tests with 4 hand-scan entries per
# lane), then an A/B of the hand scan's entries per lane and the SET append's occupancy on
# the headline (walk stream, working set = the log).
set -o pipefail
bash scripts/gpu_tests.sh r6_t2 tests/test_hbm_gpu.py tests/test_eviction.py tests/test_hot_spreading_gpu.py || exit 1
SHELLAC_RCSCAN_K=4 bash scripts/gpu_tests.sh r6_t2k4 tests/test_eviction.py -m gpu || exit 1
EXTRA="--pressured-fill 1.0 --no-cycled --overfull-fill 0" bash scripts/env_ab.sh r6_occ \
  "X=1" "SHELLAC_RCSCAN_K=2" "SHELLAC_RCSCAN_K=4" "SHELLAC_SEGOCC_1=64" "SHELLAC_SEGOCC_1=32" "X=1"
