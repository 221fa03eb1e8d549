#!/usr/bin/env bash
# Run a sequence of GPU steps on the gpurun box; stop at the first crash/timeout
# (exit >= 124, abort 134, segfault 139) but keep going after ordinary test failures.
# usage: scripts/gpu_session.sh "name:seconds:command" ...
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[gpu_session] $name rc=$rc ($(( $(date +%s) - start ))s)"
  tail -n 5 "gpurun_out/$name.log"
  if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then
    echo "[gpu_session] fatal exit in $name; stopping"
    exit "$rc"
  fi
done
