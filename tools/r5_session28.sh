#!/bin/bash
# Round-5: trace_stream waves x refill in the wavefront at the head (two-array queries, XCD bands).
set -u
export TMPDIR=/tmp
STEPS=8 bash tools/lib_matrix.sh 2 "w7r16||" "w8r16|DRT_WAVEFRONT_WAVES=8|" "w7r12|DRT_WAVEFRONT_REFILL_MIN=12|" \
  "w7r20|DRT_WAVEFRONT_REFILL_MIN=20|" "w6r16|DRT_WAVEFRONT_WAVES=6|" "w8r24|DRT_WAVEFRONT_WAVES=8 DRT_WAVEFRONT_REFILL_MIN=24|"
