#!/bin/bash
# Interleaved bench A/B over library builds and environments (no CPU baseline, no P3F leg).
# Usage: bash tools/lib_matrix.sh REPS "label|ENV=..|bench args" ...   -> gpurun_out/lib_matrix.jsonl
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT; : > $OUT/lib_matrix.jsonl
reps=$1; shift
for rep in $(seq 1 $reps); do
  for spec in "$@"; do
    IFS='|' read -r label envs args <<< "$spec"
    env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-load-timing $args \
      > $OUT/m.json 2> $OUT/m.err
    rc=$?
    python - "$label" "$envs" $OUT/m.json >> $OUT/lib_matrix.jsonl <<'PY'
import json, sys
d = json.load(open(sys.argv[3]))
print(json.dumps({"label": sys.argv[1], "env": sys.argv[2], "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "kernel_ms": d["roofline"]["kernel_ms"], "node_visits_per_ray": d["node_visits_per_ray"],
                  "bytes_per_ray": d["bytes_per_ray"], "shadow_tree": d.get("shadow_tree"), "simd_eff": d["simd_eff"],
                  "cycle_share": d["cycle_share"], "cycles_per_iter": d.get("cycles_per_iter"),
                  "passes": d["roofline"].get("passes")}))
PY
    tail -1 $OUT/lib_matrix.jsonl | cut -c1-150
    [ $rc -eq 0 ] || exit $rc
  done
done
