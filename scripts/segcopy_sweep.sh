#!/usr/bin/env bash
# Sweep the segcopy kernel variants and minimum tile sizes with kernel_bench.py.
set -u
for v in 1 6 7 2; do
  for mt in 1024; do
    printf '{"variant": %s, "min_tile": %s, "res": ' "$v" "$mt"
    SHELLAC_SEGCOPY_VARIANT=$v SHELLAC_SEGCOPY_MIN_TILE=$mt timeout -k 10 120 \
      python benchmarks/kernel_bench.py --iters 30 2>/dev/null | tail -n 1 || exit $?
    echo "}"
  done
done
