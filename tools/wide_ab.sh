#!/bin/bash
# Shadow-tree session: its parity tests, then interleaved A/B of the shadow tree on / off
# (DRT_WIDE_SHADOW) on the headline and C3, then the full GPU parity suite.  Stops at the first
# step that faults, aborts or times out.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT; : > $OUT/wide_ab.jsonl
timeout -k 10 500 python -u -m pytest tests/test_gpu_shadow_tree.py -x -v -s --timeout 300 --timeout-method thread \
  > $OUT/shadow_tree_tests.log 2>&1
rc=$?; echo "shadow-tree pytest rc=$rc"; tail -12 $OUT/shadow_tree_tests.log
if [ $rc -ge 2 ]; then exit $rc; fi
ab() {  # label, env, bench args...
  local label=$1 v=$2; shift 2
  env $v timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-load-timing "$@" > $OUT/ab.json 2> $OUT/ab.err
  local rc=$?
  python - "$label" "$v" $OUT/ab.json >> $OUT/wide_ab.jsonl <<'PY'
import json, sys
d = json.load(open(sys.argv[3]))
print(json.dumps({"label": sys.argv[1], "env": sys.argv[2], "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "kernel_ms": d["roofline"]["kernel_ms"], "frac": d["roofline"]["frac"],
                  "bytes_per_ray": d["bytes_per_ray"], "node_visits_per_ray": d["node_visits_per_ray"],
                  "shadow_tree": d.get("shadow_tree"), "simd_eff": d["simd_eff"], "cycle_share": d["cycle_share"]}))
PY
  tail -1 $OUT/wide_ab.jsonl | cut -c1-220
  return $rc
}
PK=distributionraytracer_amd/csrc/build/alt/libdrt_wpk.so  # packed-f32 wide child test (DRT_WIDE_PK)
FIRST=distributionraytracer_amd/csrc/build/alt/libdrt_wfirst.so  # first hit child, no distance order
for rep in 1 2; do
  ab headline DRT_WIDE_SHADOW=1 || exit $?
  ab headline DRT_WIDE_SHADOW=0 || exit $?
  [ -f $PK ] && { ab headline_pk DRT_LIBRARY=$PK || exit $?; }
  [ -f $FIRST ] && { ab headline_first DRT_LIBRARY=$FIRST || exit $?; }
done
for rep in 1 2; do
  ab C3 DRT_WIDE_SHADOW=1 --tris 100000 --light-spp 4 || exit $?
  ab C3 DRT_WIDE_SHADOW=0 --tris 100000 --light-spp 4 || exit $?
  [ -f $PK ] && { ab C3_pk DRT_LIBRARY=$PK --tris 100000 --light-spp 4 || exit $?; }
  [ -f $FIRST ] && { ab C3_first DRT_LIBRARY=$FIRST --tris 100000 --light-spp 4 || exit $?; }
done
if [ "${GRID:-0}" = "1" ]; then  # Grid layout experiment: inline records vs the Morton-indexed variant
  for rep in 1 2; do
    ab grid_inline DRT_WIDE_SHADOW=1 --accel grid || exit $?
    ab grid_indexed DRT_LIBRARY=distributionraytracer_amd/csrc/build/alt/libdrt_gidx.so --accel grid || exit $?
  done
fi
if [ "${C4:-1}" = "1" ]; then
  ab C4 DRT_WIDE_SHADOW=1 --res 1024 --aperture 8 --focal 1 --max-depth 8 --roughness 0.1 --steps 3 || exit $?
  ab C4 DRT_WIDE_SHADOW=0 --res 1024 --aperture 8 --focal 1 --max-depth 8 --roughness 0.1 --steps 3 || exit $?
fi
if [ "${PARITY:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "gpu pytest rc=$rc"; tail -8 $OUT/gpu_tests.log
  exit $rc
fi
