#!/bin/bash
# Round 6: Grid shadow tree — parity tests, fallback statistics, A/B (tree + grid_stream fallback /
# tree + one-thread fallback / walk), and the rocprof kernel split of a tree frame.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_grid_tree.py -x -q --timeout 300 --timeout-method thread \
  > $OUT/gv_tests.log 2>&1
rc=$?; echo "grid-tree tests rc=$rc"; tail -2 $OUT/gv_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gv_stats.py > $OUT/gv_stats.json 2> $OUT/gv_stats.err
rc=$?; echo "stats rc=$rc $(cat $OUT/gv_stats.json)"
[ $rc -eq 0 ] || { tail -5 $OUT/gv_stats.err; exit $rc; }
: > $OUT/gv_ab.jsonl
for rep in 1 2; do
  for v in ${GV_VARIANTS:-"DRT_GRID_SHADOW_TREE=1" "DRT_GRID_TREE_WIDEN_LOG2=-17" "DRT_GRID_SHADOW_TREE=0"}; do
    env $v timeout -k 10 300 python bench.py --accel grid --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline \
      > $OUT/gv_ab.json 2> $OUT/gv_ab.err
    rc=$?
    [ $rc -eq 0 ] || { tail -20 $OUT/gv_ab.err; exit $rc; }
    python - "$v" $OUT/gv_ab.json >> $OUT/gv_ab.jsonl <<'PY'
import json,sys
d=json.load(open(sys.argv[2]))
r=d["roofline"]
print(json.dumps({"variant": sys.argv[1], "config": "headline_grid", "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "passes": [{k: p.get(k) for k in ("pass", "ms", "launches")} for p in r.get("passes", [])]}))
PY
    tail -1 $OUT/gv_ab.jsonl | cut -c1-160
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/gv_prof -o gv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --accel grid --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/gv_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find $GRAFT_REPO_ROOT/$OUT/gv_prof -name '*stats*.csv' | head -3
exit $rc
