#!/bin/bash
# Round-6 probe: the GET gather staging its loads by LDS-DMA (SHELLAC_GLDS=1) vs through
# VGPRs (default): the GPU tests of the HBM cache with the LDS-DMA gather, then the bench
# alternating on one box, --check on.
set -o pipefail
SHELLAC_GLDS=1 bash scripts/gpu_tests.sh r6_glds_ab/tests tests/test_hbm_gpu.py -m gpu || exit 1
EXTRA="--no-cycled --overfull-fill 0" bash scripts/env_ab.sh r6_glds_ab \
  "X=1" "SHELLAC_GLDS=1" "X=1" "SHELLAC_GLDS=1" "X=1" "SHELLAC_GLDS=1"
