#!/bin/bash
# Routed-step iteration: GPU tests + benches (--check), then kernel/marker traces.
set -o pipefail
bash scripts/r3_routed_check.sh ${1:-r3_routed_c} && \
  TRACE_CASES="--routed;--simulate-world 8" bash scripts/r3_trace_routed.sh ${2:-r3_trace_c}
