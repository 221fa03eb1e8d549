#!/usr/bin/env bash
# A/B of the segcopy store policy (variant 1 = plain stores, 6 = nontemporal stores).
set -u
for rep in 1 2 3; do
  for v in 1 6; do
    printf '{"variant": %s, "rep": %s, "res": ' "$v" "$rep"
    SHELLAC_SEGCOPY_VARIANT=$v timeout -k 10 120 python benchmarks/kernel_bench.py --iters 100 \
      2>/dev/null | tail -n 1 || exit $?
    echo "}"
  done
done
