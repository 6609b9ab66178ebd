#!/bin/bash
# Round-5: the AA closest-chain pass writing the wavefront queries itself (DRT_WAVEFRONT_FUSED=1):
# parity with the fused pass, then the headline against the unfused pass of the same build and the
# build without the fused code (libdrt_aos.so).
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
DRT_WAVEFRONT_FUSED=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "wavefront or aa_two_pass" > $OUT/wf_tests.log 2>&1
rc=$?; tail -3 $OUT/wf_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=8 bash tools/lib_matrix.sh 2 "fused|DRT_WAVEFRONT_FUSED=1|" "unfused||" \
  "pre|DRT_LIBRARY=distributionraytracer_amd/csrc/build/alt/libdrt_aos.so|" \
  "C3_fused|DRT_WAVEFRONT_FUSED=1|--tris 100000 --light-spp 4" "C3_unfused||--tris 100000 --light-spp 4"
