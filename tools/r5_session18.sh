#!/bin/bash
# Round-5: XCD bands of the wavefront query array (DRT_WAVEFRONT_BANDS=8): parity, then A/B on the
# headline, C3 and the Grid.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "wavefront or two_pass" > $OUT/wf_tests.log 2>&1
rc=$?; tail -5 $OUT/wf_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=8 bash tools/lib_matrix.sh 2 "head_b1||" "head_b8|DRT_WAVEFRONT_BANDS=8|" "C3_b1||--tris 100000 --light-spp 4" \
  "C3_b8|DRT_WAVEFRONT_BANDS=8|--tris 100000 --light-spp 4" "grid_b1||--accel grid" "grid_b8|DRT_WAVEFRONT_BANDS=8|--accel grid"
