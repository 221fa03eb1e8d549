#!/bin/bash
# Round-6 probe: the step's cross-stream events as the kernels' own stop events
# (SHELLAC_STOP_EVENTS=1, the new default) vs marker packets (=0), alternating on one box,
# after the GPU tests that drive ShardedCache.serve; one variant with default-fence stop
# events (SHELLAC_STOP_FENCE=system).
set -o pipefail
bash scripts/gpu_tests.sh r6_stop_ab/tests tests/test_hbm_gpu.py tests/test_routed_multiproc_gpu.py -m gpu || exit 1
EXTRA="--no-cycled --overfull-fill 0" bash scripts/env_ab.sh r6_stop_ab \
  "SHELLAC_STOP_EVENTS=0" "X=1" "SHELLAC_STOP_EVENTS=0" "X=1" "SHELLAC_STOP_FENCE=system"
