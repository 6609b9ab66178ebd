#!/bin/bash
# Round-5: frames in flight (1 / 2 / 3) with the wavefront replay — headline, Grid, C3.
set -u
export TMPDIR=/tmp
STEPS=10 bash tools/lib_matrix.sh 2 "head_f1||--frames-in-flight 1" "head_f2||--frames-in-flight 2" "head_f3||--frames-in-flight 3" \
  "grid_f1||--accel grid --frames-in-flight 1" "grid_f2||--accel grid --frames-in-flight 2" \
  "C3_f1||--tris 100000 --light-spp 4 --frames-in-flight 1" "C3_f2||--tris 100000 --light-spp 4 --frames-in-flight 2"
