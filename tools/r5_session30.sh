#!/bin/bash
# Round-5: shadow-query records through the scalar cache when a wave's visiting lanes share one
# (-DDRT_UNI_FETCH, libdrt_uni.so): parity subset on that build, then headline / C3 A/B.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
UNI=DRT_LIBRARY=distributionraytracer_amd/csrc/build/alt/libdrt_uni.so
env $UNI timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow_tree.py -x -v --timeout 120 \
  --timeout-method thread -m gpu -k "wavefront or shadow or trace" > $OUT/uni_tests.log 2>&1
rc=$?; tail -3 $OUT/uni_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=8 bash tools/lib_matrix.sh 2 "head||" "head_uni|$UNI|" "C3||--tris 100000 --light-spp 4" "C3_uni|$UNI|--tris 100000 --light-spp 4"
