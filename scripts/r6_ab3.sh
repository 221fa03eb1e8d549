#!/bin/bash
# Round-6 probe: the next SET batch's log append no longer waits for this step's gather (the
# lookup reserves two batches' bytes; SHELLAC_APPEND_AHEAD=1), alternating with the default
# on one box, --check on.
set -o pipefail
EXTRA="--no-cycled --overfull-fill 0" bash scripts/env_ab.sh r6_ahead \
  "X=1" "SHELLAC_APPEND_AHEAD=1" "X=1" "SHELLAC_APPEND_AHEAD=1"
