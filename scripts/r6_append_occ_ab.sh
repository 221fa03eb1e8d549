#!/bin/bash
# Round-6 probe: the SET append (k_segcopy<1>) on a small grid that stays resident beside the
# lookup (8/64 and 16/64 of its co-resident slots: 1 and 2 workgroups per CU) vs 48/64.
set -o pipefail
EXTRA="--no-cycled --overfull-fill 0" bash scripts/env_ab.sh r6_append_occ_ab \
  "X=1" "SHELLAC_SEGOCC_1=8" "SHELLAC_SEGOCC_1=16" "X=1" "SHELLAC_SEGOCC_1=8" "SHELLAC_SEGOCC_1=16"
