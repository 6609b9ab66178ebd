#!/bin/bash
# Round-5: the streaming shadow kernel (trace_stream, 4-ary shadow tree) on 8 M-query batches of the
# bench scene's shadow rays: the rate a wavefront replay (shading split from the shadow traversal)
# would run its shadow queries at.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python tools/trace_bench.py --spp 32 --waves 6,8 --reps 3 > $OUT/trace_bench_spp32.log 2>&1
rc=$?; grep -E "^(shadow|primary|reflect)" $OUT/trace_bench_spp32.log | cut -c1-400; exit $rc
