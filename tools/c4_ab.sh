#!/bin/bash
# A/B of environment variants on the C4 workload (1M tris, 1024^2, 64 spp, DoF, glossy, depth 8),
# e.g. bash tools/c4_ab.sh "DRT_SEQ_DONATE=0" "DRT_SEQ_DONATE=1" "DRT_SEQ_SLACK=150".
# One JSON line per variant into gpurun_out/c4_ab.jsonl.  RES / STEPS override the size.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT; : > $OUT/c4_ab.jsonl
for v in "$@"; do
  env $v timeout -k 10 300 python bench.py --res ${RES:-1024} --steps ${STEPS:-3} --warmup 1 --spp 64 --aperture 8 \
      --focal 1 --max-depth 8 --roughness 0.1 --no-cpu-baseline > $OUT/c4_ab_run.json 2> $OUT/c4_ab_run.err
  rc=$?
  python - "$v" $OUT/c4_ab_run.json >> $OUT/c4_ab.jsonl <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(json.dumps({"env": sys.argv[1], "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "kernel_ms_serial": d["roofline"]["kernel_ms_serial"], "frac": d["roofline"]["frac"],
                  "simd_eff": d["simd_eff"], "rays_per_frame": d["rays_per_frame"]}))
PY
  tail -1 $OUT/c4_ab.jsonl
  [ $rc -eq 0 ] || exit $rc
done
