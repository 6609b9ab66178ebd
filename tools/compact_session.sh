#!/bin/bash
# Round-6 A/B: compact wavefront queries (WfArgs::compact, TraceArgs::sparse 2) against the thr = -1
# markers (DRT_WAVEFRONT_COMPACT=0), same library.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=8 bash tools/lib_matrix.sh 2 "compact||" "markers|DRT_WAVEFRONT_COMPACT=0|" "c3_compact||--tris 100000 --light-spp 4" \
  "c3_markers|DRT_WAVEFRONT_COMPACT=0|--tris 100000 --light-spp 4" \
  "c4_compact||--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8 --steps 3" \
  "c4_markers|DRT_WAVEFRONT_COMPACT=0|--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8 --steps 3" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/compact_ab.jsonl
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-load-timing > $OUT/compact_launch.json 2>/dev/null
