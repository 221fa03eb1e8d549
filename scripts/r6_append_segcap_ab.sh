#!/bin/bash
# Round-6 probe: the SET append with 256 staged segments per pass (4 KB of LDS instead of
# 16 KB; SHELLAC_APPEND_SEGCAP=256), so more of its workgroups fit beside the lookup.
set -o pipefail
SHELLAC_APPEND_SEGCAP=256 bash scripts/gpu_tests.sh r6_append_segcap_ab/tests tests/test_hbm_gpu.py -m gpu || exit 1
EXTRA="--no-cycled --overfull-fill 0" bash scripts/env_ab.sh r6_append_segcap_ab \
  "X=1" "SHELLAC_APPEND_SEGCAP=256" "X=1" "SHELLAC_APPEND_SEGCAP=256" "X=1" "SHELLAC_APPEND_SEGCAP=256"
