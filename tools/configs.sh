#!/bin/bash
# Every BASELINE.json configuration on one MI355X (bench.py, with the CPU baseline), one JSON
# line each into gpurun_out/configs.jsonl.  C1 (CPU-only plumbing) is the oracle/parity suite.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT; : > $OUT/configs.jsonl
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps ${CFG_STEPS:-3} --warmup 1 --cpu-seconds 8 "$@" > $OUT/cfg_$name.json 2> $OUT/cfg_$name.err
  local rc=$?
  echo "{\"config\": \"$name\", \"rc\": $rc, \"line\": $(cat $OUT/cfg_$name.json 2>/dev/null || echo null)}" >> $OUT/configs.jsonl
  echo "$name rc=$rc $(cut -c1-160 $OUT/cfg_$name.json)"
  return $rc
}
run C2_balls_low_bvh_512_16spp --scene balls_low --res 512 --spp 16 --steps 30 &&  # 1 ms frames: more steps
run C3_tri100k_512_64spp_soft4 --tris 100000 --res 512 --spp 64 --light-spp 4 &&
run headline_tri1M_512_64spp &&
run headline_grid --accel grid &&
run C4_tri1M_1024_64spp_dof_glossy_depth8 --res 1024 --spp 64 --aperture 8 --focal 1 --max-depth 8 --roughness 0.1
