#!/bin/bash
# AA two-pass sample threshold: the GPU suite, the shipped scenes' AA frames and the headline bench.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -n 2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/grid_vs_bvh.py --frames 30 --modes aa16 --scenes dragon,balls_high,assignment1 > $OUT/gvb_thr.jsonl 2> $OUT/gvb_thr.err || exit $?
python3 -c "
import json
for l in open('$OUT/gvb_thr.jsonl'):
    d=json.loads(l); print('threshold', d['scene'], d['grid']['mrays_s'], d['bvh']['mrays_s'], d['grid']['kernel_ms'], d['bvh']['kernel_ms'])
"
bash tools/lib_matrix.sh 1 "head|DRT_X=1|" "grid|DRT_X=1|--accel grid"
