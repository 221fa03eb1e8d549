#!/bin/bash
# Round-6 probe: per-stream priorities of the one-GPU step (SHELLAC_STREAM_PRIO="plan,set,asm";
# 1 = least, -1 = greatest on this image): the hand / planning stream low so its kernels
# yield freed slots to the SET chain, the SET stream high, both; alternating on one box.
set -o pipefail
EXTRA="--no-cycled --overfull-fill 0" bash scripts/env_ab.sh r6_prio_ab \
  "X=1" "SHELLAC_STREAM_PRIO=1,0,0" "SHELLAC_STREAM_PRIO=0,-1,0" "SHELLAC_STREAM_PRIO=1,-1,0" \
  "X=1" "SHELLAC_STREAM_PRIO=1,0,0" "SHELLAC_STREAM_PRIO=0,-1,0" "SHELLAC_STREAM_PRIO=1,-1,0"
