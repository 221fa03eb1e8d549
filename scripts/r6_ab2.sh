#!/bin/bash
# Round-6 batch: the moves' index pass over the window's hot rows only (k_rc_emit's list):
# the CLOCK / SET GPU tests, then an A/B against the tree before it (ab_base, a worktree of
# the previous commit) on the headline, and the pass's workgroup cap.
set -o pipefail
bash scripts/gpu_tests.sh r6_t3 tests/test_eviction.py tests/test_hbm_gpu.py tests/test_hot_spreading_gpu.py -m gpu || exit 1
AB_ARGS="--no-cycled --overfull-fill 0" bash scripts/ab_trees.sh r6_ab2 3 . ab_base || exit 1
EXTRA="--no-cycled --overfull-fill 0" bash scripts/env_ab.sh r6_mg \
  "X=1" "SHELLAC_MOVE_GRID=512" "SHELLAC_MOVE_GRID=256" "X=1"
