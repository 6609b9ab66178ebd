#!/bin/bash
# Round-5: the Grid's shadow stream with XCD bands at 7 waves; C4's in-order chain refill at 4 idle lanes.
set -u
export TMPDIR=/tmp
C4="--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8"
STEPS=6 bash tools/lib_matrix.sh 2 "grid_b1||--accel grid" "grid_b8|DRT_WAVEFRONT_BANDS=8|--accel grid" || exit $?
cp gpurun_out/lib_matrix.jsonl gpurun_out/lib_matrix_grid.jsonl
STEPS=3 bash tools/lib_matrix.sh 3 "c4_r8||$C4" "c4_r4|DRT_REFILL_MIN=4|$C4"
