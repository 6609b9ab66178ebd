#!/bin/bash
# Round-4 session: the GPU suite at the head, then bench lines (frames in flight 2 / 3, Grid) and a
# kernel trace of the Grid headline's two-pass frame.  Stops at the first failing step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -n 4 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/lib_matrix.sh 2 "head|DRT_X=1|" "head_fif3|DRT_X=1|--frames-in-flight 3" "grid|DRT_X=1|--accel grid" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_grid -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-load-timing --accel grid > $OUT/prof_grid.json 2> $OUT/prof_grid.err
rc=$?; echo "rocprof rc=$rc"; exit $rc
