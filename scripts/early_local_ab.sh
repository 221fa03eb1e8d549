#!/usr/bin/env bash
# A/B of the routed step's early local (replica) gather: right after host sync 1 on a
# third stream (SHELLAC_EARLY_LOCAL=1) vs in finish() after the reply exchange (default).
# Simulated 8 and 2 ranks, alternating, one box.
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for d in 0 1; do
    for cfg in "--simulate-world 8" "--simulate-world 2"; do
      out=$(SHELLAC_EARLY_LOCAL=$d timeout -k 10 150 python bench.py --steps 20 --warmup 5 \
            --no-smoke --no-uncoalesced --no-wrapped --check $cfg 2> gpurun_out/el_err.log) || {
        echo "FAIL early=$d $cfg"; tail -5 gpurun_out/el_err.log; exit 1; }
      chk=$(grep "check:" gpurun_out/el_err.log | tr '\n' ' ')
      echo "rep=$rep early=$d $cfg $(echo "$out" | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print("ms/step", j["ms_per_step"], "median", j.get("ms_per_step_median_gpu_events"))') $chk"
    done
  done
done
