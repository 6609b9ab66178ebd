#!/bin/bash
# Interleaved A/B of libdrt builds on the headline, C3 and C4 bench configs (no cpu baseline),
# after the BVH GPU parity tests on the in-tree build.  Usage: bash tools/lib_ab.sh LIB1 LIB2 ...
# ("base" = the in-tree libdrt.so, otherwise a path under distributionraytracer_amd/csrc/)
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scenes.py -m gpu -x -q --timeout 300 \
    > $OUT/lib_ab_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/lib_ab_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
one() {  # lib name args...
  local lib=$1 name=$2; shift 2
  local envv=""; [ "$lib" != base ] && envv="DRT_LIBRARY=$PWD/distributionraytracer_amd/csrc/$lib"
  env $envv timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline "$@" > $OUT/lab.json 2> $OUT/lab.err || return $?
  python -c "import json; d=json.load(open('$OUT/lab.json')); print(f\"{'$name':9s} {'$(basename $lib)':18s} {d['value']:8.1f} Mrays/s {d['ms_per_step']:8.2f} ms\", flush=True)"
}
for rep in $(seq ${REPS:-2}); do
  for lib in "$@"; do
    one $lib headline || exit $?
    one $lib C3 --tris 100000 --light-spp 4 || exit $?
    [ -n "${NO_C4:-}" ] || one $lib C4 --res 1024 --aperture 8 --focal 1 --max-depth 8 --roughness 0.1 || exit $?
  done
done
