#!/bin/bash
# Round-6 re-check of the byte movers' slot shares after the stop-event change: the gather
# (mode 4) and the SET append (mode 1) at 40 / 56 of 64 co-resident slots vs the default 48.
set -o pipefail
EXTRA="--no-cycled --overfull-fill 0" bash scripts/env_ab.sh r6_occ_ab \
  "X=1" "SHELLAC_SEGOCC_4=56" "SHELLAC_SEGOCC_4=40" "SHELLAC_SEGOCC_1=56" "SHELLAC_SEGOCC_1=40" \
  "X=1" "SHELLAC_SEGOCC_4=56" "SHELLAC_SEGOCC_4=40" "SHELLAC_SEGOCC_1=56" "SHELLAC_SEGOCC_1=40"
