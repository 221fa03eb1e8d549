#!/usr/bin/env bash
# Host-side profile (cProfile) of the routed step with a tiny batch: the GPU work is
# negligible, so the step time is the host's own cost (Python, bindings, collectives, syncs)
set -eu
mkdir -p gpurun_out
timeout -k 10 200 python -m cProfile -o gpurun_out/routed.prof bench.py --routed --batch 4096 \
  --sets 256 --keys-per-gpu 65536 --log-gb 1 --steps 300 --warmup 20 --no-smoke \
  --no-uncoalesced > gpurun_out/routed_prof.log 2>&1
python - <<'PY'
import pstats
p = pstats.Stats("gpurun_out/routed.prof")
p.sort_stats("tottime").print_stats(25)
PY
