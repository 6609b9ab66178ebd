#!/bin/bash
# Hit-normals record (DRT_HIT_NORMALS variant): its two-pass parity tests, then interleaved A/B on the
# headline, C3, C4 and the Grid, and the Grid's per-pass walk caps.  Stops at the first failing step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
H=distributionraytracer_amd/csrc/build/alt/libdrt_hn.so
DRT_LIBRARY=$H timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "two_pass or render_matches" --timeout 300 --timeout-method thread > $OUT/t_hn.log 2>&1
rc=$?; tail -n 3 $OUT/t_hn.log; [ $rc -eq 0 ] || exit $rc
C4="--res 1024 --aperture 8 --focal 1 --max-depth 8 --roughness 0.1 --steps 3"
G="--accel grid"
bash tools/lib_matrix.sh 2 "head|DRT_X=1|" "head_hn|DRT_LIBRARY=$H|" "c3|DRT_X=1|--tris 100000 --light-spp 4" "c3_hn|DRT_LIBRARY=$H|--tris 100000 --light-spp 4" \
  "grid|DRT_X=1|$G" "grid_hn|DRT_LIBRARY=$H|$G" "grid_w33|DRT_CHAIN_GRID_WALK=3 DRT_REPLAY_GRID_WALK=3|$G" "grid_w22|DRT_CHAIN_GRID_WALK=2 DRT_REPLAY_GRID_WALK=2|$G" \
  "grid_w32|DRT_CHAIN_GRID_WALK=3 DRT_REPLAY_GRID_WALK=2|$G" "c4|DRT_X=1|$C4" "c4_hn|DRT_LIBRARY=$H|$C4"
