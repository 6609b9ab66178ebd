#!/bin/bash
# Round 6 close: the Grid tree's parity tests at the head, its refill knob around the default, and the
# Grid headline config line (bench.py with the CPU baseline) -> gpurun_out/cfg_headline_grid.json
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_grid_tree.py -x -q --timeout 300 --timeout-method thread \
  > $OUT/gv_tests.log 2>&1
rc=$?; echo "grid-tree tests rc=$rc"; tail -2 $OUT/gv_tests.log
[ $rc -eq 0 ] || exit $rc
: > $OUT/gv_ab.jsonl
for rep in 1 2; do
  for v in DRT_GRID_TREE_REFILL_MIN=16 DRT_GRID_TREE_REFILL_MIN=24 DRT_GRID_TREE_REFILL_MIN=20; do
    env $v timeout -k 10 300 python bench.py --accel grid --steps 5 --warmup 1 --no-cpu-baseline \
      > $OUT/gv_ab.json 2> $OUT/gv_ab.err || { tail -20 $OUT/gv_ab.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$OUT/gv_ab.json')); print(json.dumps({'variant': '$v', 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" >> $OUT/gv_ab.jsonl
    tail -1 $OUT/gv_ab.jsonl
  done
done
timeout -k 10 300 python bench.py --accel grid --steps 10 --warmup 1 --cpu-seconds 8 > $OUT/cfg_headline_grid.json \
  2> $OUT/cfg_headline_grid.err
rc=$?; echo "grid config rc=$rc $(cut -c1-200 $OUT/cfg_headline_grid.json)"
exit $rc
