#!/usr/bin/env bash
# A/B of the routed step's deferred SET join (RoutedStep::join_sets): the main-shard
# SET chain of step i joined by step i+1's owner lookup (default) vs at the end of
# step i (SHELLAC_DEFER_SET_JOIN=0). Simulated 8 and 2 ranks and the one-rank RCCL
# step, alternating, one box.
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for d in 0 1; do
    for cfg in "--simulate-world 8" "--simulate-world 2" "--routed"; do
      out=$(SHELLAC_DEFER_SET_JOIN=$d timeout -k 10 150 python bench.py --steps 20 --warmup 5 \
            --no-smoke --no-uncoalesced --check $cfg 2> gpurun_out/defer_err.log) || {
        echo "FAIL defer=$d $cfg"; tail -5 gpurun_out/defer_err.log; exit 1; }
      chk=$(grep "check:" gpurun_out/defer_err.log | tr '\n' ' ')
      echo "rep=$rep defer=$d $cfg $(echo "$out" | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print("ms/step", j["ms_per_step"], "median", j.get("ms_per_step_median_gpu_events"))') $chk"
    done
  done
done
