#!/bin/bash
# Round 6: the Grid scene's shadow tree (trace_stream GV + grid_fallback) — its parity tests, the
# whole-frame Grid headline against the oracle, and an interleaved A/B of the Grid headline
# (DRT_GRID_SHADOW_TREE=1 tree / 0 walk) plus the BVH headline as a control.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_grid_tree.py -x -v --timeout 300 --timeout-method thread \
  > $OUT/gv_tests.log 2>&1
rc=$?; echo "grid-tree tests rc=$rc"; tail -4 $OUT/gv_tests.log
[ $rc -eq 0 ] || exit $rc
if [ "${GV_ORACLE:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 500 --timeout-method thread \
    -k "headline_grid" > $OUT/gv_oracle.log 2>&1
  rc=$?; echo "grid headline vs oracle rc=$rc"; tail -3 $OUT/gv_oracle.log
  [ $rc -eq 0 ] || exit $rc
fi
: > $OUT/gv_ab.jsonl
for rep in 1 2; do
  for v in "DRT_GRID_SHADOW_TREE=1" "DRT_GRID_SHADOW_TREE=0"; do
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
    tail -1 $OUT/gv_ab.jsonl | cut -c1-200
  done
done
timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > $OUT/gv_bvh.json 2> $OUT/gv_bvh.err
rc=$?; echo "bvh headline rc=$rc $(cut -c1-200 $OUT/gv_bvh.json)"
exit $rc
