#!/bin/bash
# Kernel + marker traces of the routed step (simulated 2 and 8 ranks, one-rank RCCL).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${1:-r3_trace}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export SHELLAC_TRACE=1
IFS=";" read -ra CASES <<< "${TRACE_CASES:---simulate-world 2;--simulate-world 8;--routed}"
for args in "${CASES[@]}"; do
  name=$(echo "x$args" | tr -d ' -')
  [ -n "$args" ] || name=xn1
  timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d "$OUT/$name" -o bench -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-smoke --no-uncoalesced --no-wrapped --pressured-gb 0 $args \
    > "$OUT/$name.log" 2>&1 || { echo "trace $args failed"; tail -20 "$OUT/$name.log"; exit 1; }
  f=$(find "$OUT/$name" -name '*kernel_trace.csv' | head -1)
  d=$(dirname "$f")
  for x in "$d"/*kernel_trace.csv; do [ "$(basename $x)" = bench_kernel_trace.csv ] || cp "$x" "$d/bench_kernel_trace.csv"; done
  for x in "$d"/*marker_api_trace.csv; do [ "$(basename $x)" = bench_marker_api_trace.csv ] || cp "$x" "$d/bench_marker_api_trace.csv"; done
  python3 $R/scripts/step_trace_summary.py "$d" 10 > "$OUT/${name}_summary.txt" 2>&1
  head -45 "$OUT/${name}_summary.txt"
  [ -s "$OUT/${name}_summary.txt" ] && grep -q "plan markers" "$OUT/${name}_summary.txt" && rm -rf "$OUT/$name"
done
