#!/bin/bash
# Step timelines and host-wait audits on the box, summarised there (the raw rocprofv3 CSVs of
# a HIP-API trace outgrow what gpurun copies back): `bash scripts/trace_summaries.sh OUT`.
# `bash scripts/trace_summaries.sh OUT ["n1 n1fresh pressured routed sim8"]` (N1_HIP=1: HIP API trace
# for the one-GPU runs too). Runs scripts/trace_bench.sh for the N=1 step (wrapped headline
# or fresh), the one-rank RCCL routed step and the simulated 8-rank step, writes
# step_trace_summary.py / host_wait_audit.py output under gpurun_out/OUT/, then deletes the
# raw traces.
set -o pipefail
OUT=${1:-trace_summaries}
R=gpurun_out/$OUT
mkdir -p "$R"
export TRACE_LIMIT=${TRACE_LIMIT:-240}
run() {  # name marker hip_trace bench-args...
  local name=$1 marker=$2 hip=$3
  shift 3
  HIP_TRACE=$hip TRACE_OUT=$OUT/raw_$name bash scripts/trace_bench.sh "$@" > "$R/$name.log" 2>&1 \
    || { echo "trace $name failed"; tail -20 "$R/$name.log"; return 1; }
  python3 scripts/step_trace_summary.py "gpurun_out/$OUT/raw_$name" ${TRACE_STEPS:-8} "$marker" > "$R/${name}_summary.txt"
  if [ "$hip" = 1 ]; then
    python3 scripts/host_wait_audit.py "gpurun_out/$OUT/raw_$name" 8 "$marker" > "$R/${name}_hostwait.txt"
    python3 scripts/launch_lag.py "gpurun_out/$OUT/raw_$name" 8 "$marker" > "$R/${name}_launch_lag.txt"
  fi
  rm -rf "gpurun_out/$OUT/raw_$name"
  echo "== $name"; head -3 "$R/${name}_summary.txt"
  [ "$hip" = 1 ] && head -12 "$R/${name}_hostwait.txt"
  return 0
}
WHICH=${2:-"n1 routed sim8"}
ok=0
for w in $WHICH; do
  case $w in
    n1) run n1 hbm.lookup_coalesced ${N1_HIP:-0} --no-uncoalesced --pressured-gb 0 || ok=1 ;;
    pressured) run pressured hbm.lookup_coalesced ${N1_HIP:-0} --no-uncoalesced --pressured-gb 0 --log-gb 5 || ok=1 ;;
    n1fresh) run n1fresh hbm.lookup_coalesced ${N1_HIP:-0} --no-uncoalesced --pressured-gb 0 --no-wrapped || ok=1 ;;
    routed) run routed serve.plan 1 --routed --no-uncoalesced --no-wrapped || ok=1 ;;
    sim8) run sim8 serve.plan 1 --simulate-world 8 --no-uncoalesced --no-wrapped || ok=1 ;;
  esac
  [ $ok -ne 0 ] && exit 1
done
exit 0
