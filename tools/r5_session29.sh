#!/bin/bash
# Round-5: trace_stream refill threshold 10 / 12 / 16 on the headline and C3.
set -u
export TMPDIR=/tmp
STEPS=8 bash tools/lib_matrix.sh 2 "h_r12|DRT_WAVEFRONT_REFILL_MIN=12|" "h_r10|DRT_WAVEFRONT_REFILL_MIN=10|" "h_r16||" \
  "c3_r12|DRT_WAVEFRONT_REFILL_MIN=12|--tris 100000 --light-spp 4" "c3_r16||--tris 100000 --light-spp 4"
