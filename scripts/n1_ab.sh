#!/bin/bash
# A/B of N=1 bench variants on one box: `bash scripts/n1_ab.sh OUT "ARGS1" "ARGS2" ...`
# (each ARGS a quoted string of extra bench.py flags; "" = the defaults). One JSON per
# variant under gpurun_out/OUT/, one summary line each.
set -o pipefail
OUT=gpurun_out/${1:-n1_ab}
shift
mkdir -p "$OUT"
k=0
for a in "$@"; do
  k=$((k + 1))
  timeout -k 10 300 python -u bench.py --no-uncoalesced --no-smoke $a > "$OUT/v$k.json" 2> "$OUT/v$k.err" \
    || { echo "variant $k ($a) failed"; tail -20 "$OUT/v$k.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/v$k.json')); f=d.get('log_fresh') or {}; p=d.get('log_pressured') or {}; print('v$k', repr('$a'), 'wrapped', d['ms_per_step'], 'fresh', f.get('ms_per_step'), 'pressured', p.get('ms_per_step'), 'probes/req', d['get_probes_per_request'])"
done
