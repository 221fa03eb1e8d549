#!/bin/bash
# The driver's N>1 command shape (torch.distributed.run, one process per rank) rehearsed on
# the box's one GPU: --bounce puts every rank on cuda:0 with gloo collectives. Functional
# only (N processes share one GPU; --route host is the N>1 default, which --bounce alone
# replaces by the device-routed step; the wrapped block is skipped to keep it short);
# `--check` verifies sampled GETs. Output gpurun_out/OUT.
set -o pipefail
O=gpurun_out/${1:-r6_bounce}; mkdir -p "$O"
for n in 2 4; do
  timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --bounce --route host --no-wrapped \
    --steps 5 --warmup 2 --check > "$O/bounce$n.json" 2> "$O/bounce$n.err" \
    || { echo "N=$n failed"; tail -30 "$O/bounce$n.err"; exit 1; }
  echo "N=$n: $(cut -c1-400 $O/bounce$n.json)"
  grep -h "check:" "$O/bounce$n.err" | sort | uniq -c
done
