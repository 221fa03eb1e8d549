#!/bin/bash
# N=1 bench twice (headline + secondary blocks) into gpurun_out/$1
set -o pipefail
OUT=gpurun_out/${1:-r3_ab}
mkdir -p "$OUT"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-smoke > "$OUT/bench$i.json" 2> "$OUT/bench$i.err" \
    || { echo "bench failed"; tail -20 "$OUT/bench$i.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench$i.json'));print(d['ms_per_step'],'wrapped',d['log_wrapped']['ms_per_step'],'pressured',d['log_pressured']['ms_per_step'],d['log_pressured']['owner_hit_ratio'],'unco',d['uncoalesced_ops_per_s'])"
done
