#!/bin/bash
# A/B several libdrt builds across the bench configurations (no cpu baseline, no parity run).
# Usage: bash tools/ab_cfg.sh LIB1 LIB2 ...   ("base" = the in-tree libdrt.so)
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
one() {  # lib, name, bench args...
  local lib=$1 name=$2; shift 2
  local envv=""; [ "$lib" != base ] && envv="DRT_LIBRARY=$lib"
  env $envv timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline "$@" \
    > $OUT/abc.json 2> $OUT/abc.err || return $?
  python -c "import json,sys; d=json.load(open('$OUT/abc.json')); print(f\"{'$name':10s} {'$(basename $lib)':24s} {d['value']:8.1f} Mrays/s {d['ms_per_step']:8.2f} ms\")"
}
for lib in "$@"; do
  one $lib headline && one $lib grid --accel grid && one $lib C3 --tris 100000 --res 512 --spp 64 --light-spp 4 &&
  one $lib C4 --res 1024 --spp 64 --aperture 8 --focal 1 --max-depth 8 --roughness 0.1 || exit $?
done
