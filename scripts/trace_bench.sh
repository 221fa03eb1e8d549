#!/usr/bin/env bash
# Timeline of the bench step: ROCTX phase ranges (SHELLAC_TRACE=1) + kernel trace.
# No PMC counters here (gpurun refuses --pmc together with marker tracing).
set -eu
cd /tmp && export TMPDIR=/tmp
OUT="${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/trace"
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export SHELLAC_TRACE=1
rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d "$OUT" -o bench -- \
  python3 bench.py --steps 10 --warmup 2 --no-smoke "$@"
