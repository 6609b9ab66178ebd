#!/bin/bash
# Round-5: bench line (one frame in flight on one GPU) and the rocprofv3 kernel trace of the same
# command, at the wavefront head.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
S=20; W=5
timeout -k 10 600 python bench.py --steps $S --warmup $W > $OUT/bench.json 2> $OUT/bench.err || exit $?
cut -c1-300 $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps $S --warmup $W --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || exit $?
python tools/rocprof_union.py $OUT/prof --steps $S --warmup $W --bench-json $OUT/prof_bench.json > $OUT/rocprof_union.json || exit $?
cat $OUT/rocprof_union.json
