#!/bin/bash
# Round-5: C4's closest-chain pass (MODE_SKEL, in-order) knobs with the wavefront replay: refill and
# shading thresholds.
set -u
export TMPDIR=/tmp
C4="--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8"
STEPS=3 bash tools/lib_matrix.sh 2 "base||$C4" "r16|DRT_REFILL_MIN=16|$C4" "r4|DRT_REFILL_MIN=4|$C4" \
  "p8|DRT_SKEL_PROCESS_MIN=8|$C4" "p40|DRT_SKEL_PROCESS_MIN=40|$C4" "chunk8M|DRT_WAVEFRONT_CHUNK_SLOTS=8388608|$C4" \
  "chunk32M|DRT_WAVEFRONT_CHUNK_SLOTS=33554432|$C4"
