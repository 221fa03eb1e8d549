#!/bin/bash
# Per-N replica size sweep of the simulated routed step (docs/PERF.md, replica table):
# `bash scripts/replica_sweep.sh OUT "N..." "R..." [extra bench args]`.
set -o pipefail
OUT=gpurun_out/${1:-replica_sweep}
WORLDS=${2:-"2 4 8"}
REPS=${3:-"0 524288 1048576 2097152 4194304"}
shift 3 || true
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for w in $WORLDS; do
  for r in $REPS; do
    f="$OUT/sim${w}_rep${r}.json"
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-uncoalesced --no-wrapped \
      --no-smoke --simulate-world "$w" --replicate "$r" "$@" > "$f" 2> "$OUT/sim${w}_rep${r}.err" \
      || { echo "sim $w rep $r failed"; tail -20 "$OUT/sim${w}_rep${r}.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$f')); print('sim$w rep $r', d['ms_per_step'], d.get('ms_per_step_median_gpu_events'), 'replica_hit', d['replica_hit_fraction'])"
  done
done
