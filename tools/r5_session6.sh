#!/bin/bash
# Round-5: replay-pass writes with the frame heads in global memory (head) against scratch (hscr),
# PMC WRITE_SIZE of the timed replay dispatch on the headline and C4; then the one-primitive leaf
# step in the replay pass (rleaf1: vector-memory read instructions per frame should drop) A/B.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
A=distributionraytracer_amd/csrc/build/alt
C4="--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8"
LIBS="base $A/libdrt_hscr.so" BENCH_ARGS="--settle-s 0 --no-load-timing" PMC_OUT=$OUT/pmc_w_head bash tools/pmc_ab.sh "WRITE_SIZE" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" > $OUT/pmc_writes_headline.jsonl || exit $?
cat $OUT/pmc_writes_headline.jsonl | cut -c1-300
LIBS="base $A/libdrt_hscr.so" BENCH_ARGS="--settle-s 0 --no-load-timing $C4" PMC_OUT=$OUT/pmc_w_c4 bash tools/pmc_ab.sh "WRITE_SIZE" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" > $OUT/pmc_writes_c4.jsonl || exit $?
cat $OUT/pmc_writes_c4.jsonl | cut -c1-300
STEPS=5 bash tools/lib_matrix.sh 2 "head|DRT_X=1|" "rleaf1|DRT_LIBRARY=$A/libdrt_rleaf1.so|" "hscr|DRT_LIBRARY=$A/libdrt_hscr.so|" \
  "c3|DRT_X=1|--tris 100000 --light-spp 4" "c3_rleaf1|DRT_LIBRARY=$A/libdrt_rleaf1.so|--tris 100000 --light-spp 4" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/ab_r5_s6.jsonl
