#!/bin/bash
# Round-6 A/B: the 8-ary shadow tree (-DDRT_WIDE8, 128-B records) against the 4-ary default.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
W8=DRT_LIBRARY=distributionraytracer_amd/csrc/build/alt/libdrt_w8.so
env $W8 timeout -k 10 600 python -u -m pytest tests/test_gpu_shadow_tree.py tests/test_gpu_parity.py -x -q --timeout 300 \
  --timeout-method thread -m gpu > $OUT/w8_tests.log 2>&1
rc=$?; tail -2 $OUT/w8_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=5 bash tools/lib_matrix.sh 2 "w4||" "w8|$W8|" "c3_w4||--tris 100000 --light-spp 4" "c3_w8|$W8|--tris 100000 --light-spp 4" \
  "c4_w4||--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8 --steps 3" \
  "c4_w8|$W8|--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8 --steps 3" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/w8_ab.jsonl
