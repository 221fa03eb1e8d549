#!/usr/bin/env bash
# A/B: SET index insert ordered by an event on the main stream (SHELLAC_HOST_ORDER=0) vs
# queued after the host read the lookup total (1); three interleaved rounds + --check
set -u
for r in 1 2 3; do
  for v in 0 1; do
    out=$(SHELLAC_HOST_ORDER=$v timeout -k 10 120 python bench.py --no-smoke --no-uncoalesced 2>/dev/null) || exit $?
    echo "round $r host_order=$v $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("ms_per_step_median_gpu_events"))')"
  done
done
SHELLAC_HOST_ORDER=1 timeout -k 10 120 python bench.py --no-smoke --no-uncoalesced --check 2>&1 | grep check
