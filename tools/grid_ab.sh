#!/bin/bash
# Grid stepper A/B on the 1M-triangle headline scene with `accel grid`: the Grid parity tests
# first, then interleaved bench runs of each variant ("LIB|ENV..." with LIB "base" = the in-tree
# libdrt.so).  Usage: bash tools/grid_ab.sh "base|DRT_GRID_PAIRS=3" "build/alt/libdrt_x.so|" ...
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "grid" --timeout 300 \
    > $OUT/grid_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/grid_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq ${REPS:-2}); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    lib=${v%%|*}; envs=${v#*|}
    envv=""; [ "$lib" != base ] && envv="DRT_LIBRARY=$PWD/distributionraytracer_amd/csrc/$lib"
    env $envv $envs timeout -k 10 300 python bench.py --accel grid --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline \
      > $OUT/gab_$i.json 2> $OUT/gab_$i.err
    rc=$?
    python - "$v" $OUT/gab_$i.json <<'PY'
import json,sys
try:
    d=json.load(open(sys.argv[2])); print(f"{sys.argv[1]:56s} {d['value']:8.1f} Mrays/s {d['ms_per_step']:8.2f} ms  simd={d.get('simd_eff')}", flush=True)
except Exception as e: print(sys.argv[1], 'FAILED', e, flush=True)
PY
    [ $rc -eq 0 ] || exit $rc
  done
done
