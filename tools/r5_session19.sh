#!/bin/bash
# Round-5: per-kernel times of C4 and the Grid headline at the wavefront head (rocprofv3 kernel trace).
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --settle-s 0 --no-cpu-baseline --no-load-timing --res 1024 --aperture 8 --focal 1 \
  --roughness 0.1 --max-depth 8 > $OUT/prof_c4.json 2> $OUT/prof_c4.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_grid -o run --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 --settle-s 0 --no-cpu-baseline --no-load-timing --accel grid > $OUT/prof_grid.json 2> $OUT/prof_grid.err || exit $?
head -8 $OUT/prof_c4/run_kernel_stats.csv | cut -c1-160
head -8 $OUT/prof_grid/run_kernel_stats.csv | cut -c1-160
