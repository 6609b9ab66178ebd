#!/bin/bash
# MODE_SEQ tail probe: the C4 workload (DoF + glossy depth 8, a lane runs a pixel's 64 samples in
# order) at 1024^2 and at 2048^2.  A lane holds ~2.7 pixels of a 1024^2 frame and ~11 of a 2048^2
# one, so a frame tail of lanes finishing their last pixel at different times shows up as a higher
# Mrays/s at 2048^2.  One JSON line per run into gpurun_out/c4_tail.jsonl.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT; : > $OUT/c4_tail.jsonl
C4="--spp 64 --aperture 8 --focal 1 --max-depth 8 --roughness 0.1 --no-cpu-baseline --warmup 1"
for cfg in "--res 1024 --steps 3" "--res 2048 --steps 2" "--res 1024 --steps 3 --frames-in-flight 1"; do
  timeout -k 10 300 python bench.py $C4 $cfg > $OUT/c4_tail_run.json 2> $OUT/c4_tail_run.err
  rc=$?
  python - "$cfg" $OUT/c4_tail_run.json >> $OUT/c4_tail.jsonl <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(json.dumps({"args": sys.argv[1], "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "kernel_ms_serial": d["roofline"]["kernel_ms_serial"], "simd_eff": d["simd_eff"],
                  "rays_per_frame": d["rays_per_frame"]}))
PY
  tail -1 $OUT/c4_tail.jsonl
  [ $rc -eq 0 ] || exit $rc
done
