#!/bin/bash
# Round-5: the AA closest-chain pass's refill / shading thresholds re-checked with the wavefront replay.
set -u
export TMPDIR=/tmp
STEPS=8 bash tools/lib_matrix.sh 2 "base||" "cp4|DRT_CHAIN_PROCESS_MIN=4|" "cp12|DRT_CHAIN_PROCESS_MIN=12|" \
  "cr4|DRT_CHAIN_REFILL_MIN=4|" "cr12|DRT_CHAIN_REFILL_MIN=12|" "cw7|DRT_CHAIN_WAVES=7|"
