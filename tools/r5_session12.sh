#!/bin/bash
# Round-5: wavefront replay, streaming-kernel waves x refill threshold on the headline (interleaved).
set -u
export TMPDIR=/tmp
STEPS=5 bash tools/lib_matrix.sh 2 "w7r24|DRT_WAVEFRONT_WAVES=7|" "w7r8|DRT_WAVEFRONT_WAVES=7 DRT_WAVEFRONT_REFILL_MIN=8|" \
  "w7r16|DRT_WAVEFRONT_WAVES=7 DRT_WAVEFRONT_REFILL_MIN=16|" "w8r8|DRT_WAVEFRONT_WAVES=8 DRT_WAVEFRONT_REFILL_MIN=8|" \
  "w8r16|DRT_WAVEFRONT_WAVES=8 DRT_WAVEFRONT_REFILL_MIN=16|" "w7r4|DRT_WAVEFRONT_WAVES=7 DRT_WAVEFRONT_REFILL_MIN=4|"
