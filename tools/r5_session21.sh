#!/bin/bash
# Round-5: the Grid wavefront's MODE_QSTREAM knobs (empty cells walked per call, object pairs per call,
# waves) on the Grid headline.
set -u
export TMPDIR=/tmp
STEPS=6 bash tools/lib_matrix.sh 1 "w3p3||--accel grid" "w5p3|DRT_REPLAY_GRID_WALK=5|--accel grid" \
  "w8p3|DRT_REPLAY_GRID_WALK=8|--accel grid" "w3p2|DRT_REPLAY_GRID_PAIRS=2|--accel grid" \
  "w3p5|DRT_REPLAY_GRID_PAIRS=5|--accel grid" "w5p5|DRT_REPLAY_GRID_WALK=5 DRT_REPLAY_GRID_PAIRS=5|--accel grid" \
  "w3p3_r16|DRT_WAVEFRONT_GRID_REFILL_MIN=16|--accel grid" "w3p3_r4|DRT_WAVEFRONT_GRID_REFILL_MIN=4|--accel grid"
