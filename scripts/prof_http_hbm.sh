#!/usr/bin/env bash
# rocprofv3 kernel trace of the proxy's HBM batch path under HTTP load: HBM-only backend,
# 1M objects x 4 KiB, c=1000 (the load generator and origin are child processes; the
# proxy and its GPU batcher run in the traced Python process)
set -eu
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$R/gpurun_out/prof_http"; mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o http -- \
  python3 "$R/benchmarks/http_bench.py" --backend hbm --objects 1000000 --requests 1000000 \
  --conc 1000 --timeout 300 --out "$OUT/http.json" > "$OUT/http.log" 2>&1
grep "\[http\]" "$OUT/http.log" | cut -c1-200
