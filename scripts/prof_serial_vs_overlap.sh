#!/usr/bin/env bash
# Kernel traces of the N=1 step with the SET chain on a side stream (default) and serial
# (SHELLAC_OVERLAP_STORE=0: every kernel alone on one stream -> standalone durations)
set -eu
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
for mode in overlap serial; do
  OUT="$R/gpurun_out/step_$mode"; mkdir -p "$OUT"
  if [ $mode = serial ]; then export SHELLAC_OVERLAP_STORE=0; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o bench -- \
    python3 "$R/bench.py" --steps 10 --warmup 2 --no-smoke --no-uncoalesced > "$OUT/bench.log" 2>&1
  tail -1 "$OUT/bench.log" | cut -c1-160
done
