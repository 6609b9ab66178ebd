#!/bin/bash
# Round-5: wavefront replay (wf_gen + trace_stream + wf_combine) — parity against the persistent
# MODE_AREPLAY pass and the reference-order frame, then an interleaved A/B on the headline and C3.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "wavefront or whitted_two_pass or aa_two_pass or refraction_two_pass or pass_times" > $OUT/wf_tests.log 2>&1
rc=$?; tail -15 $OUT/wf_tests.log; [ $rc -eq 0 ] || exit $rc
STEPS=5 bash tools/lib_matrix.sh 2 "wf|DRT_WAVEFRONT=1|" "areplay|DRT_WAVEFRONT=0|" \
  "C3_wf|DRT_WAVEFRONT=1|--tris 100000 --light-spp 4" "C3_areplay|DRT_WAVEFRONT=0|--tris 100000 --light-spp 4"
