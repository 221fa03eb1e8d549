#!/bin/bash
# A/B of N=1 bench variants that differ by environment: `bash scripts/env_ab.sh OUT "ENV1" "ENV2" ...`
# (each ENV a quoted list of VAR=value; "X=1" = the defaults), in order, one box, --check on.
set -o pipefail
O=gpurun_out/${1:-env_ab}; shift; mkdir -p "$O"
k=0
for e in "$@"; do
  k=$((k + 1))
  env $e timeout -k 10 240 python -u bench.py --no-uncoalesced --no-smoke --check > "$O/v$k.json" 2> "$O/v$k.err" \
    || { echo "variant $k ($e) failed"; tail -5 "$O/v$k.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/v$k.json')); print('v$k', repr('$e'), 'wrapped', d['ms_per_step'], 'fresh', d['log_fresh']['ms_per_step'], 'pressured', (d.get('log_pressured') or {}).get('ms_per_step'))"
  grep -h "check:" "$O/v$k.err" | tr '\n' ' '; echo
done
