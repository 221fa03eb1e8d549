#!/bin/bash
# HTTP A/B of whole source trees (each built in place): `bash scripts/http_ab_trees.sh OUT
# ROUNDS DIR... -- http_bench args`; alternating, one box.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-http_ab}; ROUNDS=${2:-2}; shift 2
DIRS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do DIRS+=("$1"); shift; done
shift
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for d in "${DIRS[@]}"; do
    tag=$(basename "$(cd "$d" && pwd)"); [ "$d" = "." ] && tag=main
    (cd "$d" && timeout -k 10 400 python benchmarks/http_bench.py "$@" --out "$OUT/${tag}_$r.json" \
       > "$OUT/${tag}_$r.log" 2>&1) || { echo "$tag $r failed"; tail -5 "$OUT/${tag}_$r.log"; exit 1; }
    grep "\[http\].*c=" "$OUT/${tag}_$r.log" | sed "s|^|$tag $r |" | cut -c1-150
  done
done
