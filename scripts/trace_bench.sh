#!/usr/bin/env bash
# Timeline of the bench step: ROCTX phase ranges (SHELLAC_TRACE=1) + kernel trace, and with
# HIP_TRACE=1 the HIP runtime calls too (for scripts/host_wait_audit.py). Output in
# gpurun_out/${TRACE_OUT:-trace}. No PMC counters here (gpurun refuses --pmc together with
# tracing). `bash scripts/trace_bench.sh [bench args]`
set -eu
cd /tmp && export TMPDIR=/tmp
# (the tree to trace: TRACE_TREE, default the repo root; the output always lands under the
# repo root's gpurun_out, which gpurun copies back)
OUT="${GRAFT_REPO_ROOT:-/root/repo}/gpurun_out/${TRACE_OUT:-trace}"
mkdir -p "$OUT"
cd "${TRACE_TREE:-${GRAFT_REPO_ROOT:-/root/repo}}"
export SHELLAC_TRACE=1
EXTRA=""
if [ "${HIP_TRACE:-0}" = 1 ]; then EXTRA="--hip-trace"; fi
timeout -k 10 ${TRACE_LIMIT:-300} rocprofv3 --marker-trace --kernel-trace $EXTRA --stats --output-format csv -d "$OUT" -o bench -- \
  python3 bench.py --steps 10 --warmup 2 --no-smoke "$@"
