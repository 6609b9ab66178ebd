#!/bin/bash
# Round-5 A/B: the head against the round-4 library and against variants that revert one change each
# (DRT_WIDE_EXACT: the two-op-per-plane shadow-tree child test; DRT_GRID_RECS48: 48-B Grid records).
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
A=distributionraytracer_amd/csrc/build/alt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow_tree.py -x -q -k "two_pass or whitted or grid or shadow" --timeout 300 --timeout-method thread > $OUT/t_s3.log 2>&1
rc=$?; tail -n 2 $OUT/t_s3.log; [ $rc -eq 0 ] || exit $rc
STEPS=5 bash tools/lib_matrix.sh 2 "head|DRT_X=1|" "r4|DRT_LIBRARY=$A/libdrt_r4.so|" "wexact|DRT_LIBRARY=$A/libdrt_wexact.so|" \
  "grid|DRT_X=1|--accel grid" "grid_r4|DRT_LIBRARY=$A/libdrt_r4.so|--accel grid" "grid_recs48|DRT_LIBRARY=$A/libdrt_recs48.so|--accel grid" \
  "c3|DRT_X=1|--tris 100000 --light-spp 4" "c3_wexact|DRT_LIBRARY=$A/libdrt_wexact.so|--tris 100000 --light-spp 4" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/ab_r5_s3.jsonl
