#!/bin/bash
# Per-rank step of the host-routed N-rank bench, simulated on one GPU (rank 0's owner share
# of the Zipf stream on its 1/N of the key space): `bash scripts/host_route_sim.sh OUT "2 4 8"`.
# The driver's defaults otherwise (wrapped headline, pressured window); --check on each.
set -o pipefail
OUT=gpurun_out/${1:-host_route_sim}
mkdir -p "$OUT"
for n in ${2:-"2 4 8"}; do
  timeout -k 10 400 python -u bench.py --no-uncoalesced --no-smoke --check --simulate-world "$n" \
    --route host > "$OUT/sim${n}.json" 2> "$OUT/sim${n}.err" \
    || { echo "sim $n failed"; tail -20 "$OUT/sim${n}.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/sim${n}.json')); f=d.get('log_fresh') or {}; p=d.get('log_pressured') or {}; print('sim$n host', 'wrapped', d['ms_per_step'], 'fresh', f.get('ms_per_step'), 'pressured', p.get('ms_per_step'), 'hit', d['get_hit_ratio'])"
  grep "check" "$OUT/sim${n}.err"
done
