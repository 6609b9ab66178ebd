#!/bin/bash
# Round-5: waves/SIMD of the Grid's wavefront passes (chain 5 / 6 / 7, MODE_QSTREAM 5 / 6 / 7).
set -u
export TMPDIR=/tmp
STEPS=6 bash tools/lib_matrix.sh 2 "c5q5||--accel grid" "c5q7|DRT_WAVEFRONT_GRID_WAVES=7|--accel grid" \
  "c6q5|DRT_CHAIN_WAVES=6|--accel grid" "c7q5|DRT_CHAIN_WAVES=7|--accel grid" \
  "c6q7|DRT_CHAIN_WAVES=6 DRT_WAVEFRONT_GRID_WAVES=7|--accel grid"
