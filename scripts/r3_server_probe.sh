#!/bin/bash
# Doorbell placement probe (host memory vs fine-grained VRAM written through the BAR).
# Runs last in a GPU call: a host segfault on the BAR write would end the call.
set -o pipefail
OUT=gpurun_out/${1:-r3_server}
mkdir -p "$OUT"
timeout -k 10 60 benchmarks/native/bin/doorbell_probe > "$OUT/doorbell_probe.log" 2>&1
rc=$?
cat "$OUT/doorbell_probe.log"
exit $rc
