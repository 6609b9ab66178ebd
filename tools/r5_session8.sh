#!/bin/bash
# Round-5: new GPU tests (per-pass times, shipped glass AA frames), then the uniform material / light
# table reads (utab: scalar loads when a wave's lanes read <= 2 distinct entries; predicted to lower the
# replay pass's vector-memory read instructions) and the AA closest-chain pass without a one-primitive
# leaf step's last-slot load (cl2: fewer lane accesses, same instructions) A/B against the head.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
A=distributionraytracer_amd/csrc/build/alt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenes.py -x -q -k "pass_times or glass or refraction" --timeout 300 --timeout-method thread > $OUT/t_s8.log 2>&1
rc=$?; tail -n 2 $OUT/t_s8.log; [ $rc -eq 0 ] || exit $rc
DRT_LIBRARY=$A/libdrt_utab.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "render_matches or two_pass or whitted or refraction" --timeout 300 --timeout-method thread > $OUT/t_s8_utab.log 2>&1
rc=$?; tail -n 2 $OUT/t_s8_utab.log; [ $rc -eq 0 ] || exit $rc
LIBS="base $A/libdrt_utab.so" BENCH_ARGS="--settle-s 0 --no-load-timing" PMC_OUT=$OUT/pmc_utab bash tools/pmc_ab.sh "SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_VALU" > $OUT/pmc_utab.jsonl || exit $?
cut -c1-300 $OUT/pmc_utab.jsonl
C4="--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8"
STEPS=5 bash tools/lib_matrix.sh 2 "head|DRT_X=1|" "utab|DRT_LIBRARY=$A/libdrt_utab.so|" "cl2|DRT_LIBRARY=$A/libdrt_cl2.so|" \
  "c3|DRT_X=1|--tris 100000 --light-spp 4" "c3_utab|DRT_LIBRARY=$A/libdrt_utab.so|--tris 100000 --light-spp 4" "c3_cl2|DRT_LIBRARY=$A/libdrt_cl2.so|--tris 100000 --light-spp 4" \
  "grid|DRT_X=1|--accel grid" "grid_utab|DRT_LIBRARY=$A/libdrt_utab.so|--accel grid" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/ab_r5_s8.jsonl
STEPS=3 bash tools/lib_matrix.sh 1 "c4|DRT_X=1|$C4" "c4_utab|DRT_LIBRARY=$A/libdrt_utab.so|$C4" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/ab_r5_s8_c4.jsonl
