#!/usr/bin/env bash
# A/B of the fence scope of the events ordering the step's two streams
# (SHELLAC_EVENT_FENCE=system: torch's events; device: hipEventReleaseToDevice;
# none: hipEventDisableSystemFence), two interleaved rounds on one box, plus --check runs
set -u
for r in 1 2; do
  for f in system device none; do
    out=$(SHELLAC_EVENT_FENCE=$f timeout -k 10 120 python bench.py --no-smoke --no-uncoalesced 2>/dev/null) || exit $?
    echo "round $r fence=$f $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_median_gpu_events"])')"
  done
done
for f in device none; do
  SHELLAC_EVENT_FENCE=$f timeout -k 10 120 python bench.py --no-smoke --no-uncoalesced --check 2>&1 | grep check
done
