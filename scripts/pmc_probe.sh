#!/usr/bin/env bash
# PMC passes over the coalescing micro-benchmark (Zipf batch): what bounds k_probe and
# k_coalesce — HBM bytes, L2 hit rate, address-translation misses. One counter group per
# run (hardware limits per block), --kernel-trace only (no tracing domains with --pmc).
set -eu
cd /tmp && export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/pmcp"
mkdir -p "$OUT"
run() {  # name, then rocprofv3 options
  local name=$1
  shift
  timeout -s KILL 120 rocprofv3 --kernel-trace "$@" --output-format csv -d "$OUT" -o "$name" -- \
    python3 "$ROOT/scripts/coalesce_micro.py" --dist zipf
}
run fetch --pmc FETCH_SIZE --kernel-include-regex "probe|coalesce"
run tcc --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "probe|coalesce"
run utcl --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --kernel-include-regex "probe|coalesce"
run sq --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "probe|coalesce"
