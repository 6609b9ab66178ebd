#!/bin/bash
# Round-5: wavefront replay with compact light-pair slots, and on the Grid (MODE_QSTREAM): parity, then
# an interleaved A/B on the Grid headline, the headline and C3.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "wavefront or whitted_two_pass or aa_two_pass or pass_times" > $OUT/wf_tests.log 2>&1
rc=$?; tail -15 $OUT/wf_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=5 bash tools/lib_matrix.sh 2 "grid_wf||--accel grid" "grid_persist|DRT_WAVEFRONT_GRID=0|--accel grid" \
  "grid_wf_w6|DRT_WAVEFRONT_GRID_WAVES=6|--accel grid" "head||" "C3||--tris 100000 --light-spp 4"
