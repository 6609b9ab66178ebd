#!/bin/bash
# Round-5: the wavefront replay's launches under rocprofv3 (per-kernel time of one headline frame),
# then its streaming-kernel knobs (waves per SIMD, refill threshold) A/B on the headline.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_wf -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-load-timing > $OUT/prof_wf.json 2> $OUT/prof_wf.err || exit $?
python tools/rocprof_union.py $OUT/prof_wf --steps 5 --warmup 1 --bench-json $OUT/prof_wf.json > $OUT/prof_wf_union.json || exit $?
cat $OUT/prof_wf_union.json
STEPS=5 bash tools/lib_matrix.sh 1 "w6r24||" "w8r24|DRT_WAVEFRONT_WAVES=8|" "w7r24|DRT_WAVEFRONT_WAVES=7|" \
  "w6r8|DRT_WAVEFRONT_REFILL_MIN=8|" "w6r40|DRT_WAVEFRONT_REFILL_MIN=40|" "w8r40|DRT_WAVEFRONT_WAVES=8 DRT_WAVEFRONT_REFILL_MIN=40|"
