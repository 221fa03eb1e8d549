#!/usr/bin/env bash
# k_coalesce cost of the global claim table: kernel stats of the coalescing micro-benchmark
# with the global table (default) and chunk-local collapsing only (SHELLAC_COALESCE_LOCAL=1)
set -eu
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
for mode in global local; do
  OUT="$R/gpurun_out/co_$mode"; mkdir -p "$OUT"
  if [ $mode = local ]; then export SHELLAC_COALESCE_LOCAL=1; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o micro -- \
    python3 "$R/scripts/coalesce_micro.py" --dist zipf > "$OUT/micro.log" 2>&1
  grep micro "$OUT/micro.log" | tail -2
done
