#!/usr/bin/env bash
# MFMA counters of the hello kernel (BASELINE.json: "single HIP MFMA 'hello' kernel on
# one MI355X with rocprof counter capture"). One counter group per run, --kernel-trace
# only (no tracing domains with PMC), each run under its own kill timeout.
set -eu
cd /tmp && export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/mfma"
mkdir -p "$OUT"
cd "$ROOT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
grep -oE "SQ_[A-Z0-9_]*MFMA[A-Z0-9_]*" "$OUT/avail.txt" | sort -u > "$OUT/mfma_counters.txt" || true
run() {  # name, counters...
  local name=$1
  shift
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc "$@" --kernel-include-regex mfma \
    --output-format csv -d "$OUT" -o "$name" -- python3 scripts/mfma_hello_run.py 4096
}
timeout -s KILL 60 rocprofv3 --kernel-trace --kernel-include-regex mfma --output-format csv -d "$OUT" -o time -- python3 scripts/mfma_hello_run.py 4096
for c in SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA; do
  run "pmc_$c" "$c" || echo "counter $c failed"
done
