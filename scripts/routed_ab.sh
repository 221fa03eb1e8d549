#!/bin/bash
# A/B of routed-step variants on one GPU: `bash scripts/routed_ab.sh OUT "variant args"...`
# Each variant runs the simulated 8- and 2-rank steps and the one-rank RCCL step.
set -o pipefail
OUT=gpurun_out/${1:-routed_ab}
shift
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for v in "$@"; do
  for args in "--simulate-world 8" "--simulate-world 2" "--routed"; do
    name=$(echo "x$args$v" | tr -d ' -')
    timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-uncoalesced --no-wrapped \
      --no-smoke $args $v > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" \
      || { echo "bench $args $v failed"; tail -30 "$OUT/bench_$name.err"; exit 1; }
    echo "== $args $v: $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_$name.json')); print(d['ms_per_step'], d.get('ms_per_step_median_gpu_events'))")"
  done
done
