#!/bin/bash
# Round-5: waves/SIMD of the in-order closest-chain pass (C4, MODE_SKEL: DRT_WAVES) and of the one-pass
# AA frame (C2).
set -u
export TMPDIR=/tmp
C4="--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8"
STEPS=3 bash tools/lib_matrix.sh 2 "c4_w6||$C4" "c4_w7|DRT_WAVES=7|$C4" "c2_w6||--scene balls_low --spp 16 --steps 30" \
  "c2_w7|DRT_WAVES=7|--scene balls_low --spp 16 --steps 30"
