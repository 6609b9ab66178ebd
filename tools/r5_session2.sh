#!/bin/bash
# Round-5 session: the GPU suite at the head (one-fma shadow-tree child test, Whitted two-pass frames,
# 40-B Grid triangle pairs), then interleaved A/B against the round-4 library and the shipped Grid
# scenes' Whitted / AA frames.  Stops at the first failing step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -n 4 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
R4=distributionraytracer_amd/csrc/build/alt/libdrt_r4.so
STEPS=5 bash tools/lib_matrix.sh 2 "head|DRT_X=1|" "r4|DRT_LIBRARY=$R4|" "grid|DRT_X=1|--accel grid" "grid_r4|DRT_LIBRARY=$R4|--accel grid" \
  "c3|DRT_X=1|--tris 100000 --light-spp 4" "c3_r4|DRT_LIBRARY=$R4|--tris 100000 --light-spp 4" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/ab_r5_s2.jsonl
timeout -k 10 400 python tools/grid_vs_bvh.py --frames 20 --modes whitted > $OUT/gvb_whitted_head.jsonl 2> $OUT/gvb.err
rc=$?; echo "gvb head rc=$rc"; [ $rc -eq 0 ] || exit $rc
DRT_LIBRARY=$R4 timeout -k 10 400 python tools/grid_vs_bvh.py --frames 20 --modes whitted > $OUT/gvb_whitted_r4.jsonl 2> $OUT/gvb_r4.err
rc=$?; echo "gvb r4 rc=$rc"; exit $rc
