#!/usr/bin/env bash
# A/B of the side-stream SET overlap and the gather's share of co-resident slots
# (SHELLAC_OVERLAP_STORE x SHELLAC_SEGCOPY_OCC) on the N=1 bench step.
set -u
mkdir -p gpurun_out
for ov in ${OVS:-0 1 2}; do
  for occ in ${OCCS:-48}; do
    r=$(SHELLAC_OVERLAP_STORE=$ov SHELLAC_SEGCOPY_OCC=$occ timeout -k 10 120 \
        python bench.py --steps 30 --warmup 5 --no-smoke "$@" 2>/dev/null) || exit $?
    echo "overlap=$ov occ=$occ $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], round(d["value"]/1e9,3))')"
  done
done
