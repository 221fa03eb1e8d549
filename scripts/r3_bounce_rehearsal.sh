#!/bin/bash
# The multi-GPU bench flow on one GPU: N ranks (torchrun child launch), the native routed
# executor with its collectives bounced through gloo (functional, not a performance
# number), --check ground truth on every rank's last batch.
set -o pipefail
OUT=gpurun_out/${1:-r3_bounce}
mkdir -p "$OUT"
for n in 2 4; do
  timeout -k 10 420 python -u bench.py --gpus $n --bounce --steps 4 --warmup 3 --check \
    --no-uncoalesced --no-wrapped --pressured-gb 0 --keys-per-gpu 1048576 --log-gb 4 \
    > "$OUT/bounce$n.json" 2> "$OUT/bounce$n.err" \
    || { echo "bounce $n failed"; tail -30 "$OUT/bounce$n.err"; exit 1; }
  echo "== $n ranks"; grep "check" "$OUT/bounce$n.err"; cut -c1-260 "$OUT/bounce$n.json"
done
