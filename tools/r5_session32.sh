#!/bin/bash
# Round-5: the AA closest-chain pass at 7 waves/SIMD — headline and C3, with its refill / shading thresholds.
set -u
export TMPDIR=/tmp
STEPS=8 bash tools/lib_matrix.sh 2 "h_w6||" "h_w7|DRT_CHAIN_WAVES=7|" "h_w7_p12|DRT_CHAIN_WAVES=7 DRT_CHAIN_PROCESS_MIN=12|" \
  "h_w7_r12|DRT_CHAIN_WAVES=7 DRT_CHAIN_REFILL_MIN=12|" "c3_w6||--tris 100000 --light-spp 4" \
  "c3_w7|DRT_CHAIN_WAVES=7|--tris 100000 --light-spp 4"
