#!/usr/bin/env bash
# HBM traffic of the hot cache kernels (kernel_bench.py workload): FETCH_SIZE and
# WRITE_SIZE (KiB to/from HBM) per dispatch -- one counter per run, the pair exceeds
# what the hardware collects in one pass -- joined with the kernel durations of a plain
# kernel-trace run by scripts/pmc_summary.py. PMC runs use --kernel-trace only.
set -eu
cd /tmp && export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
cd "$ROOT"
run() {  # name, then rocprofv3 options
  local name=$1
  shift
  timeout -k 10 150 rocprofv3 --kernel-trace "$@" --output-format csv -d "$OUT" -o "$name" -- \
    python3 benchmarks/kernel_bench.py --iters 3
}
run fetch --pmc FETCH_SIZE --kernel-include-regex "segcopy|probe|set_index|set_dedupe"
run write --pmc WRITE_SIZE --kernel-include-regex "segcopy|probe|set_index|set_dedupe"
run occ --pmc SQ_WAVES SQ_BUSY_CYCLES --kernel-include-regex "segcopy|probe"
run time
