#!/bin/bash
# Round-6 A/B: the Grid's wavefront shadow queries on grid_stream (compact queries) against the path
# kernel's MODE_QSTREAM over the marker layout (DRT_GRID_STREAM=0), same library.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
G="--accel grid"
STEPS=6 bash tools/lib_matrix.sh 2 "gs||$G" "qstream|DRT_GRID_STREAM=0|$G" "gs_b8|DRT_WAVEFRONT_BANDS=8|$G" \
  "gs_w6|DRT_WAVEFRONT_GRID_WAVES=6|$G" "gs_w5|DRT_WAVEFRONT_GRID_WAVES=5|$G" "gs_r8|DRT_WAVEFRONT_GRID_REFILL_MIN=8|$G" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/gstream_ab.jsonl
