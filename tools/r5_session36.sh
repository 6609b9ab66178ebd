#!/bin/bash
# Round-5: C4's wavefront chunk size (2^24 default, 2^25, 2^26: 4 / 2 / 1 chunks).
set -u
export TMPDIR=/tmp
C4="--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8"
STEPS=3 bash tools/lib_matrix.sh 3 "c24||$C4" "c25|DRT_WAVEFRONT_CHUNK_SLOTS=33554432|$C4" "c26|DRT_WAVEFRONT_CHUNK_SLOTS=67108864|$C4"
