#!/bin/bash
# Round-5: wavefront replay for in-order (DoF / glossy) frames and in chunks: parity, then C4 and the
# headline A/B (wavefront vs the persistent replay).
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "wavefront or two_pass or pass_times" > $OUT/wf_tests.log 2>&1
rc=$?; tail -12 $OUT/wf_tests.log; [ $rc -eq 0 ] || exit $rc
C4="--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8"
STEPS=3 bash tools/lib_matrix.sh 1 "C4_wf||$C4" "C4_persist|DRT_WAVEFRONT_INORDER=0|$C4" "head||" \
  "head_chunk4M|DRT_WAVEFRONT_CHUNK_SLOTS=4194304|"
