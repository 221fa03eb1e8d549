#!/usr/bin/env bash
# PMC counters for the cache kernels (no tracing domains besides kernel trace).
set -eu
cd /tmp && export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
cd "$ROOT"
rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "segcopy|probe|set_index" --output-format csv -d "$OUT" -o pmc1 -- \
  python3 benchmarks/kernel_bench.py --iters 3
rocprofv3 --kernel-trace --pmc FETCH_SIZE TA_BUSY_avr \
  --kernel-include-regex "segcopy|probe" --output-format csv -d "$OUT" -o pmc2 -- \
  python3 benchmarks/kernel_bench.py --iters 3
