#!/bin/bash
# Round-5: the Grid wavefront's MODE_QSTREAM refill threshold, and the Grid chain pass's.
set -u
export TMPDIR=/tmp
STEPS=6 bash tools/lib_matrix.sh 2 "r16|DRT_WAVEFRONT_GRID_REFILL_MIN=16|--accel grid" \
  "r24|DRT_WAVEFRONT_GRID_REFILL_MIN=24|--accel grid" "r32|DRT_WAVEFRONT_GRID_REFILL_MIN=32|--accel grid" \
  "r48|DRT_WAVEFRONT_GRID_REFILL_MIN=48|--accel grid" \
  "r24_c16|DRT_WAVEFRONT_GRID_REFILL_MIN=24 DRT_CHAIN_REFILL_MIN=16|--accel grid" \
  "r24_w6|DRT_WAVEFRONT_GRID_REFILL_MIN=24 DRT_WAVEFRONT_GRID_WAVES=6|--accel grid"
