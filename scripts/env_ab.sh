#!/bin/bash
# A/B of N=1 bench variants that differ by environment: `bash scripts/env_ab.sh OUT "ENV1" "ENV2" ...`
# (each ENV a quoted list of VAR=value; "X=1" = the defaults), in order, one box, --check on.
# EXTRA: extra bench.py flags for every variant.
set -o pipefail
O=gpurun_out/${1:-env_ab}; shift; mkdir -p "$O"
k=0
for e in "$@"; do
  k=$((k + 1))
  env $e timeout -k 10 300 python -u bench.py --no-uncoalesced --no-smoke --check $EXTRA > "$O/v$k.json" 2> "$O/v$k.err" \
    || { echo "variant $k ($e) failed"; tail -5 "$O/v$k.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/v$k.json')); p=d.get('log_pressured') or {}; w=d.get('log_wrapped') or {}
print('v$k', repr('$e'), d['headline_phase'], d['ms_per_step'], 'fresh', d['log_fresh']['ms_per_step'], 'wrapped', w.get('ms_per_step'), 'pressured', p.get('ms_per_step'), 'lap', p.get('lap_ms_per_step'), 'hit', p.get('owner_hit_ratio'))"
  grep -h "check:" "$O/v$k.err" | tr '\n' ' '; echo
done
