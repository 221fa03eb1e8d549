#!/usr/bin/env bash
# Grid-size sweep of k_probe / k_coalesce on the coalescing micro-benchmark (Zipf):
# per-kernel average GPU time (rocprofv3 --kernel-trace --stats) for each grid cap.
set -eu
cd /tmp && export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out/gsweep"
mkdir -p "$OUT"
for g in 2048 1024 512 256; do
  SHELLAC_PROBE_GRID=$g SHELLAC_COALESCE_GRID=$((g / 2)) timeout -k 10 120 \
    rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/g$g" -o m -- \
    python3 "$ROOT/scripts/coalesce_micro.py" --dist zipf > "$OUT/g$g.log" 2>&1
  python3 - "$OUT/g$g/m_kernel_stats.csv" "$g" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_probe" in r["Name"] or "k_coalesce" in r["Name"]:
        print(f"grid {sys.argv[2]:>5} {r['Name'][:45]:45s} avg {float(r['AverageNs'])/1e3:7.1f} us")
PY
done
