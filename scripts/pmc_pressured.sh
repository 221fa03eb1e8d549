#!/bin/bash
# PMC passes over the pressured step (a 4.92 GiB log, the default working set 0.8 of it):
# HBM bytes of every dispatch of the byte movers and the CLOCK hand, one counter group per
# run (FETCH_SIZE, WRITE_SIZE), listed per dispatch by scripts/pmc_dispatches.py.
# `bash scripts/pmc_pressured.sh OUT [bench args]`. Counter collection serialises the
# dispatches: the trace of these runs gives each kernel's time alone.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P=gpurun_out/${1:-pmc_pressured}; shift
mkdir -p "$P"
ARGS="--steps 40 --warmup 2 --no-uncoalesced --no-smoke --pressured-gb 0 --log-gb 4.92 $*"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $P/$c -o run -- python3 bench.py $ARGS > $P/$c.log 2>&1 || { tail -5 $P/$c.log; exit 1; }
done
for k in "k_segcopy<1" "k_segcopy<0" k_rc_emit k_rc_scan k_coalesce; do
  python3 scripts/pmc_dispatches.py $P "$k" 45 > "$P/$(echo $k | tr -c 'a-z0-9_\n' '_').txt"
done
python3 - "$P" <<'PY'
import csv, glob, os, sys
d = sys.argv[1]
for f in glob.glob(os.path.join(d, "FETCH_SIZE", "**", "*kernel_trace.csv"), recursive=True):
    rows = [r for r in csv.DictReader(open(f)) if "k_segcopy<1" in r["Kernel_Name"]]
    ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows][-45:]
    print("k_segcopy<1> alone (us), last 45:", " ".join(f"{x:.0f}" for x in ds))
PY
rm -rf $P/FETCH_SIZE $P/WRITE_SIZE
