#!/bin/bash
# A/B: hardware queues per process (HIP default 4) for the routed step's streams.
set -o pipefail
OUT=gpurun_out/${1:-r3_hwq_ab}
mkdir -p "$OUT"
for q in 4 8 4 8; do
  for args in "--routed" "--simulate-world 8"; do
    name=$(echo "q${q}$args" | tr -d ' -')
    GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-uncoalesced \
      --no-wrapped --pressured-gb 0 --no-smoke $args > "$OUT/$name.json" 2> "$OUT/$name.err" \
      || { echo "bench $q $args failed"; tail -20 "$OUT/$name.err"; exit 1; }
    echo "q=$q $args $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(d['ms_per_step'], d.get('ms_per_step_median_gpu_events'))")"
  done
done
