#!/bin/bash
# The most loaded rank of the host-routed N-rank job, simulated on one GPU (its true share of
# the global Zipf stream on its 1/N of the key space), with hot-object spreading off and on:
# `bash scripts/host_route_sim.sh OUT "2 4 8" ["0 1024"]`. The driver's defaults otherwise
# (the pressured headline); --check on each. SIM_ARGS: extra bench flags.
set -o pipefail
OUT=gpurun_out/${1:-host_route_sim}
mkdir -p "$OUT"
for n in ${2:-"2 4 8"}; do
  for k in ${3:-"0 1024"}; do
    tag=sim${n}_spread${k}
    timeout -k 10 400 python -u bench.py --no-uncoalesced --no-smoke --check --simulate-world "$n" \
      --route host --spread "$k" $SIM_ARGS > "$OUT/$tag.json" 2> "$OUT/$tag.err" \
      || { echo "$tag failed"; tail -20 "$OUT/$tag.err"; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/$tag.json')); f=d.get('log_fresh') or {}; w=d.get('log_wrapped') or {}; p=d.get('log_pressured') or {}; h=d['host_routing']
print('$tag rank', h['simulated_rank'], 'share max/mean', h['rank_share_max_over_mean'], d['headline_phase'], d['ms_per_step'], 'lap', p.get('lap_ms_per_step'), 'fresh', f.get('ms_per_step'), 'wrapped', w.get('ms_per_step'), 'hit', d['get_hit_ratio'], 'request hit', p.get('request_hit_ratio'), 'router', h['host_route_req_per_s'], h['host_route_threads'], 'thr', h['host_route_req_per_s_one_thread'], 'feeds', h.get('router_feeds_job'))"
    grep "check" "$OUT/$tag.err"
  done
done
