#!/bin/bash
# Round-6 A/B: the shadow-tree child decode in trace_stream — one fma per plane (-DDRT_WIDE_FMA1) and
# packed-f32 pairs (-DDRT_WIDE_PK) against the reference arithmetic (default).
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
F1=DRT_LIBRARY=distributionraytracer_amd/csrc/build/alt/libdrt_fma1.so
PK=DRT_LIBRARY=distributionraytracer_amd/csrc/build/alt/libdrt_pk.so
env $F1 timeout -k 10 600 python -u -m pytest tests/test_gpu_shadow_tree.py tests/test_gpu_parity.py -x -q --timeout 300 \
  --timeout-method thread -m gpu -k "shadow or wavefront or trace or render" > $OUT/fma1_tests.log 2>&1
rc=$?; tail -2 $OUT/fma1_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=5 bash tools/lib_matrix.sh 2 "def||" "fma1|$F1|" "pk|$PK|" "c3_def||--tris 100000 --light-spp 4" \
  "c3_fma1|$F1|--tris 100000 --light-spp 4" "c3_pk|$PK|--tris 100000 --light-spp 4" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/decode_ab.jsonl
