#!/bin/bash
# GPU tests on one MI355X under one time limit: `bash scripts/gpu_tests.sh OUT [pytest args]`.
# Default: the whole GPU suite. Output under gpurun_out/OUT/.
set -o pipefail
OUT=gpurun_out/${1:-gpu_tests}
shift || true
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(tests -m gpu)
timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread "${ARGS[@]}" \
  > "$OUT/tests.log" 2>&1
rc=$?
tail -5 "$OUT/tests.log"
[ $rc -ne 0 ] && grep -E "FAILED|Error|error" "$OUT/tests.log" | head -20
exit $rc
