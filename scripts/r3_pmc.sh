#!/bin/bash
# Round-3 PMC rooflines: the N=1 step and the one-rank routed step (headline steps only).
set -o pipefail
PMC_OUT=gpurun_out/r3_pmc_n1 bash scripts/pmc_roofline.sh --no-wrapped --pressured-gb 0 && \
PMC_OUT=gpurun_out/r3_pmc_routed bash scripts/pmc_roofline.sh --no-wrapped --pressured-gb 0 --routed
