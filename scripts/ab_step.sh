#!/usr/bin/env bash
# A/B of the N=1 step schedules on one box: SHELLAC_COMPACT x SHELLAC_PLAN_FIRST, two
# interleaved rounds (boxes differ by several %, so only same-call numbers compare).
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for c in 0 1; do
    for p in 0 1; do
      out=$(SHELLAC_COMPACT=$c SHELLAC_PLAN_FIRST=$p timeout -k 10 120 python bench.py --no-smoke \
            --no-uncoalesced "$@" 2>/dev/null) || exit $?
      ms=$(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_median_gpu_events"])')
      echo "round $r compact=$c plan_first=$p ms/step(wall, gpu-median) $ms"
    done
  done
done
