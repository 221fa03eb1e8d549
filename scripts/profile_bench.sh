#!/usr/bin/env bash
# Kernel-level profile of the bench step: rocprofv3 kernel trace + stats (no PMC).
set -eu
cd /tmp && export TMPDIR=/tmp
OUT="${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/prof"
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o bench -- \
  python3 bench.py --steps 10 --warmup 2 --no-smoke "$@"
