#!/bin/bash
# Headline full-cache block on the walk stream at several --pressured-fill values (working
# set over the log): request hit ratio, read working set per lap, ms/step.
# `bash scripts/fill_sweep.sh OUT fill...`
set -o pipefail
OUT=gpurun_out/${1:-fill_sweep}
shift
mkdir -p "$OUT"
for f in "$@"; do
  timeout -k 10 400 python -u bench.py --pressured-fill "$f" --no-cycled --overfull-fill 0 \
    --no-uncoalesced > "$OUT/fill_$f.json" 2> "$OUT/fill_$f.err" \
    || { echo "fill $f failed"; tail -20 "$OUT/fill_$f.err"; exit 1; }
  python - "$OUT/fill_$f.json" "$f" <<'PY'
import json, sys
o = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = o["log_pressured"]
print(f"fill {sys.argv[2]}: ms {p['ms_per_step']} (gpu {p.get('ms_per_step_median_gpu_events')}) "
      f"lap {p['lap_ms_per_step']} req_hit {p['request_hit_ratio']} owner_hit {p['owner_hit_ratio']} "
      f"read_ws {p['read_working_set_over_capacity']} reins {p['reinserted_bytes_per_step_per_rank']}")
PY
done
