#!/bin/bash
# Round-5: the GPU suite at the head (exact shadow-tree decode, MODE_AREPLAY, BVH replay frame heads
# in lane-contiguous global memory, 40-B Grid triangle pairs), then A/B against the round-4 library
# and the head with scratch frame heads (hscr).
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
A=distributionraytracer_amd/csrc/build/alt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -n 3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
C4="--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8"
STEPS=5 bash tools/lib_matrix.sh 2 "head|DRT_X=1|" "r4|DRT_LIBRARY=$A/libdrt_r4.so|" "hscr|DRT_LIBRARY=$A/libdrt_hscr.so|" \
  "grid|DRT_X=1|--accel grid" "grid_r4|DRT_LIBRARY=$A/libdrt_r4.so|--accel grid" \
  "c3|DRT_X=1|--tris 100000 --light-spp 4" "c3_r4|DRT_LIBRARY=$A/libdrt_r4.so|--tris 100000 --light-spp 4" "c3_hscr|DRT_LIBRARY=$A/libdrt_hscr.so|--tris 100000 --light-spp 4" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/ab_r5_s5.jsonl
STEPS=3 bash tools/lib_matrix.sh 1 "c4|DRT_X=1|$C4" "c4_r4|DRT_LIBRARY=$A/libdrt_r4.so|$C4" "c4_hscr|DRT_LIBRARY=$A/libdrt_hscr.so|$C4" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/ab_r5_s5_c4.jsonl
