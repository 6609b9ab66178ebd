#!/bin/bash
# Round-5: after the fused-chain revert (wf_gen on the shared wf_level helper): parity subset, and the
# headline / Grid against the build before the fusion experiment (libdrt_aos.so).
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "wavefront or two_pass" > $OUT/wf_tests.log 2>&1
rc=$?; tail -3 $OUT/wf_tests.log; [ $rc -eq 0 ] || exit $rc
PRE=DRT_LIBRARY=distributionraytracer_amd/csrc/build/alt/libdrt_aos.so
STEPS=8 bash tools/lib_matrix.sh 2 "head||" "head_pre|$PRE|" "C3||--tris 100000 --light-spp 4" "C3_pre|$PRE|--tris 100000 --light-spp 4"
