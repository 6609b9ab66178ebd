#!/bin/bash
# Round-5: wavefront query validity from per-sample level counts (no empty-slot markers): parity subset,
# then headline / C3 / Grid / C4 against the marker build (libdrt_aos.so).
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenes.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "wavefront or two_pass or pass_times or shipped" > $OUT/wf_tests.log 2>&1
rc=$?; tail -3 $OUT/wf_tests.log; [ $rc -eq 0 ] || exit $rc
PRE=DRT_LIBRARY=distributionraytracer_amd/csrc/build/alt/libdrt_aos.so
C4="--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8"
STEPS=8 bash tools/lib_matrix.sh 2 "head||" "head_pre|$PRE|" "C3||--tris 100000 --light-spp 4" "C3_pre|$PRE|--tris 100000 --light-spp 4" \
  "grid||--accel grid" "grid_pre|$PRE|--accel grid" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/lib_matrix_a.jsonl
STEPS=3 bash tools/lib_matrix.sh 2 "C4||$C4" "C4_pre|$PRE|$C4"
