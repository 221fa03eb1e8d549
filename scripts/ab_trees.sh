#!/bin/bash
# A/B of whole source trees on one box: `bash scripts/ab_trees.sh OUT ROUNDS DIR...` runs the
# driver's N=1 bench (no uncoalesced block, no smoke) from each tree DIR in turn (each built
# in place beforehand, e.g. a git worktree of a variant), ROUNDS times, alternating. One JSON
# per (round, tree) under gpurun_out/OUT/ and a summary line each.
set -o pipefail
OUT=${1:-ab_trees}
ROUNDS=${2:-2}
shift 2
R=$GRAFT_REPO_ROOT/gpurun_out/$OUT
mkdir -p "$R"
for r in $(seq 1 "$ROUNDS"); do
  for d in "$@"; do
    tag=$(basename "$(cd "$d" && pwd)")
    [ "$d" = "." ] && tag=main
    (cd "$d" && timeout -k 10 300 python -u bench.py --no-uncoalesced --no-smoke $AB_ARGS \
       > "$R/${tag}_$r.json" 2> "$R/${tag}_$r.err") \
      || { echo "$tag round $r failed"; tail -20 "$R/${tag}_$r.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$R/${tag}_$r.json')); f=d.get('log_fresh') or {}; p=d.get('log_pressured') or {}; print('$tag', $r, 'wrapped', d['ms_per_step'], 'fresh', f.get('ms_per_step'), 'pressured', p.get('ms_per_step'))"
  done
done
