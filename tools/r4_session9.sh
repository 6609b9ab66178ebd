#!/bin/bash
# AA two-pass frame-time rule: the GPU suite, the shipped scenes' AA frames (one at a time), and the
# 1M / C3 scenes at 16 and 64 spp (pipelined) with the rule and with two passes forced.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -n 2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/grid_vs_bvh.py --frames 30 --modes aa16 --scenes dragon,balls_high,assignment1 > $OUT/gvb_rule.jsonl 2> $OUT/gvb_rule.err || exit $?
python3 -c "
import json
for l in open('$OUT/gvb_rule.jsonl'):
    d=json.loads(l); print('rule', d['scene'], d['grid']['mrays_s'], d['bvh']['mrays_s'], d['grid']['kernel_ms'], d['bvh']['kernel_ms'])
"
bash tools/lib_matrix.sh 1 "head|DRT_X=1|" "spp16|DRT_X=1|--spp 16" "spp16_2p|DRT_AA_TWO_PASS_MIN_MS=0|--spp 16" "spp16_1p|DRT_AA_TWO_PASS=0|--spp 16" "c3spp16|DRT_X=1|--spp 16 --tris 100000 --light-spp 4" "grid|DRT_X=1|--accel grid"
