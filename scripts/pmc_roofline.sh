# PMC roofline of the N=1 bench step: per-kernel HBM bytes (FETCH_SIZE, WRITE_SIZE: one
# pass each, they cannot share the 4 TCC counters) plus a plain kernel-trace pass for
# the durations. Summarised by scripts/pmc_roofline.py into profiles/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P=${PMC_OUT:-gpurun_out/pmc}
mkdir -p "$P"
ARGS="--steps 6 --warmup 2 --no-uncoalesced --no-smoke $*"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $P/trace -o run -- python3 bench.py $ARGS > $P/trace.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- python3 bench.py $ARGS > $P/fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- python3 bench.py $ARGS > $P/write.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $P/sq -o run -- python3 bench.py $ARGS > $P/sq.log 2>&1 || exit 1
python3 scripts/pmc_roofline.py "$P" > $P/roofline.md && cat $P/roofline.md
