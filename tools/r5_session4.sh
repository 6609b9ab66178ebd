#!/bin/bash
# Round-5 A/B with the AA / Whitted replay as its own instantiation (MODE_AREPLAY): the head against
# the round-4 library, the exact two-op decode (wexact) and the 48-B Grid records (recs48); C4 too.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
A=distributionraytracer_amd/csrc/build/alt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow_tree.py -x -q -k "two_pass or whitted or grid or shadow or render_matches" --timeout 300 --timeout-method thread > $OUT/t_s4.log 2>&1
rc=$?; tail -n 2 $OUT/t_s4.log; [ $rc -eq 0 ] || exit $rc
C4="--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8"
STEPS=5 bash tools/lib_matrix.sh 2 "head|DRT_X=1|" "r4|DRT_LIBRARY=$A/libdrt_r4.so|" "wexact|DRT_LIBRARY=$A/libdrt_wexact.so|" "hscratch|DRT_LIBRARY=$A/libdrt_hscratch.so|" \
  "grid|DRT_X=1|--accel grid" "grid_r4|DRT_LIBRARY=$A/libdrt_r4.so|--accel grid" "grid_recs48|DRT_LIBRARY=$A/libdrt_recs48.so|--accel grid" "grid_hscratch|DRT_LIBRARY=$A/libdrt_hscratch.so|--accel grid" \
  "c3|DRT_X=1|--tris 100000 --light-spp 4" "c3_r4|DRT_LIBRARY=$A/libdrt_r4.so|--tris 100000 --light-spp 4" "c3_wexact|DRT_LIBRARY=$A/libdrt_wexact.so|--tris 100000 --light-spp 4" "c3_hscratch|DRT_LIBRARY=$A/libdrt_hscratch.so|--tris 100000 --light-spp 4" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/ab_r5_s4.jsonl
STEPS=3 bash tools/lib_matrix.sh 1 "c4|DRT_X=1|$C4" "c4_r4|DRT_LIBRARY=$A/libdrt_r4.so|$C4" "c4_wexact|DRT_LIBRARY=$A/libdrt_wexact.so|$C4" "c4_hscratch|DRT_LIBRARY=$A/libdrt_hscratch.so|$C4" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/ab_r5_s4_c4.jsonl
