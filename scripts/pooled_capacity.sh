#!/bin/bash
# Pooled capacity (the reference's "glue together extra memory", README.md:3/:12): a FIXED
# total key space (--keys-total, default 32M keys, ~34 GB of records) over N shards whose
# logs are a fixed size each (--pressured-gb, default 8 GiB: large enough for the hand's lead
# mode, layout.h hand_lead), so the working set is ~3.9x one
# shard's log at N = 1 and fits from N = 4 on. Each run is the most loaded rank of the
# host-routed N-rank job simulated on one GPU (N = 1: the plain one-GPU step); the full-cache
# block's SETs walk every key the rank holds (--set-walk), so an evicted key comes back when
# re-SET. Prints hit ratios (distinct keys per batch, and requests over K untimed steps) and ms.
# `bash scripts/pooled_capacity.sh OUT ["1 2 4 8"]`; KEYS / LOG_GB / CAP_ARGS override.
set -o pipefail
OUT=gpurun_out/${1:-pooled_capacity}
mkdir -p "$OUT"
KEYS=${KEYS:-33554432}
LOG_GB=${LOG_GB:-8}
for n in ${2:-"1 2 4 8"}; do
  tag=cap_n${n}
  if [ "$n" = 1 ]; then sim=""; else sim="--simulate-world $n --route host"; fi
  timeout -k 10 600 python -u bench.py --no-uncoalesced --no-smoke --keys-total "$KEYS" \
    --pressured-gb "$LOG_GB" --log-gb 2 --set-walk $sim $CAP_ARGS \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { echo "$tag failed"; tail -20 "$OUT/$tag.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$tag.json')); p=d['log_pressured']
print('$tag keys', d['config']['keys_total'], 'ws/capacity', p['working_set_over_capacity'], 'hit (distinct)', p['owner_hit_ratio'], 'hit (requests)', p.get('request_hit_ratio'), 'ms', p['ms_per_step'], 'lap', p.get('lap_ms_per_step'), 'reinserted MB', round(p['reinserted_bytes_per_step_per_rank'] / 1e6, 1), 'fill', p.get('fill_steps'))"
done
