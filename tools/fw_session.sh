#!/bin/bash
# Round-6 A/B: wf_gen with whole-wave query stores (-DDRT_WF_FULLWAVE) against the default.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
FW=DRT_LIBRARY=distributionraytracer_amd/csrc/build/alt/libdrt_fw.so
env $FW timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "wavefront or two_pass or render or full_size" > $OUT/fw_tests.log 2>&1
rc=$?; tail -2 $OUT/fw_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=8 bash tools/lib_matrix.sh 2 "def||" "fw|$FW|" "c3_def||--tris 100000 --light-spp 4" "c3_fw|$FW|--tris 100000 --light-spp 4" \
  "c4_def||--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8 --steps 3" \
  "c4_fw|$FW|--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8 --steps 3" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/fw_ab.jsonl
# per-launch times of the last serial frame (bench.py roofline.passes launches)
for v in def fw; do
  e=""; [ $v = fw ] && e=$FW
  env $e timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-load-timing > $OUT/fw_launch_$v.json 2>/dev/null || exit $?
done
