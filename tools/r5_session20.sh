#!/bin/bash
# Round-5: two-array query records (SoA) in the wavefront: parity subset, then A/B against the previous
# build (libdrt_aos.so) on the headline, C3 and the Grid; then per-kernel times of C4 and the Grid.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow_tree.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "wavefront or two_pass or trace or shadow" > $OUT/wf_tests.log 2>&1
rc=$?; tail -4 $OUT/wf_tests.log; [ $rc -eq 0 ] || exit $rc
AOS=DRT_LIBRARY=distributionraytracer_amd/csrc/build/alt/libdrt_aos.so
STEPS=8 bash tools/lib_matrix.sh 2 "head_soa||" "head_aos|$AOS|" "C3_soa||--tris 100000 --light-spp 4" \
  "C3_aos|$AOS|--tris 100000 --light-spp 4" "grid_soa||--accel grid" "grid_aos|$AOS|--accel grid" || exit $?
bash tools/r5_session19.sh
