#!/bin/bash
# Round-5: MODE_QSTREAM's re-claim of empty slots: Grid parity subset, then A/B against the build
# without it (both at refill 16).
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "wavefront or two_pass" > $OUT/wf_tests.log 2>&1
rc=$?; tail -3 $OUT/wf_tests.log; [ $rc -eq 0 ] || exit $rc
OLD="DRT_LIBRARY=distributionraytracer_amd/csrc/build/alt/libdrt_aos.so DRT_WAVEFRONT_GRID_REFILL_MIN=16"
STEPS=6 bash tools/lib_matrix.sh 2 "grid_reclaim||--accel grid" "grid_old|$OLD|--accel grid" \
  "c4grid_reclaim||--accel grid --res 256 --aperture 8 --roughness 0.1 --max-depth 8"
