#!/bin/bash
# Round-5: Grid chain and MODE_QSTREAM at 7 waves by default — the GPU suite's Grid / two-pass / scene
# tests, then the Grid headline A/B against the previous defaults.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenes.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "grid or two_pass or wavefront or whitted or shipped" > $OUT/grid_w7_tests.log 2>&1
rc=$?; tail -3 $OUT/grid_w7_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=6 bash tools/lib_matrix.sh 2 "c7q7||--accel grid" "c7q5|DRT_WAVEFRONT_GRID_WAVES=5|--accel grid" \
  "c5q5|DRT_CHAIN_WAVES=5 DRT_WAVEFRONT_GRID_WAVES=5|--accel grid" "head||"
