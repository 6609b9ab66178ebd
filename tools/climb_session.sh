#!/bin/bash
# Round-6 A/B: wavefront shadow queries that start at their hit's leaf record and climb (TraceArgs::start)
# against the root walk (DRT_SHADOW_CLIMB=0), same library: parity tests, then headline / C3 / C4.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
bash tools/session.sh "tests:climb or wavefront or shadow_tree or node_record" || exit $?
C3="--tris 100000 --light-spp 4"
C4="--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8"
STEPS=6 bash tools/lib_matrix.sh 2 "climb||" "root|DRT_SHADOW_CLIMB=0|" "climb_c3||$C3" "root_c3|DRT_SHADOW_CLIMB=0|$C3" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/climb_ab.jsonl
STEPS=3 bash tools/lib_matrix.sh 1 "climb_c4||$C4" "root_c4|DRT_SHADOW_CLIMB=0|$C4" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/climb_ab_c4.jsonl
