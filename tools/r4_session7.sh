#!/bin/bash
# Shipped Grid-default scenes' 16-spp AA frames with the AA two-pass frame on and off (both accelerators).
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
for v in 1 0 1 0; do
  DRT_AA_TWO_PASS=$v DRT_AA_TWO_PASS_GRID=$v timeout -k 10 300 python tools/grid_vs_bvh.py --frames 30 --modes aa16 \
    --scenes dragon,balls_high,assignment1 > $OUT/gvb_2p$v.jsonl 2> $OUT/gvb_2p$v.err || exit $?
  python3 -c "
import json,sys
for l in open('$OUT/gvb_2p$v.jsonl'):
    d=json.loads(l); print('two_pass=$v', d['scene'], d['grid']['mrays_s'], d['bvh']['mrays_s'], d['grid']['kernel_ms'], d['bvh']['kernel_ms'])
" | tee -a $OUT/gvb_ab.txt
done
