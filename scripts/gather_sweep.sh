# N=1 step time under segcopy occupancy / variant knobs (one box, one call)
set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 120 env "$@" python bench.py --steps 20 --warmup 5 --no-smoke --no-uncoalesced 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | sed "s|^|$* |"; }
run SHELLAC_SEGCOPY_OCC=48
run SHELLAC_SEGCOPY_OCC=64
run SHELLAC_SEGCOPY_OCC=40
run SHELLAC_SEGCOPY_VARIANT=0
run SHELLAC_SEGCOPY_VARIANT=2
run SHELLAC_SEGCOPY_VARIANT=4
run SHELLAC_SEGCOPY_VARIANT=6
run SHELLAC_SEGCOPY_VARIANT=7
run SHELLAC_SEGCOPY_MIN_TILE=2048
run SHELLAC_SEGCOPY_MIN_TILE=4096
