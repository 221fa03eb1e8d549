#!/bin/bash
# Round-6 probe: the SET index insert ordered after the lookup by a device word the lookup's
# last workgroup writes (SHELLAC_WAIT_WORDS=1; hipStreamWaitValue64 on the SET stream) instead
# of the coalescing kernel's stop event (no packet between the lookup and the gather on the
# main stream). The serve GPU tests with it first, then the bench alternating, --check on.
set -o pipefail
SHELLAC_WAIT_WORDS=1 bash scripts/gpu_tests.sh r6_words_ab/tests tests/test_hbm_gpu.py -k serve -m gpu || exit 1
EXTRA="--no-cycled --overfull-fill 0" bash scripts/env_ab.sh r6_words_ab \
  "X=1" "SHELLAC_WAIT_WORDS=1" "X=1" "SHELLAC_WAIT_WORDS=1" "X=1" "SHELLAC_WAIT_WORDS=1"
