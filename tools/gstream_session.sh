#!/bin/bash
# Round-6 grid_stream sessions.
#   A: the Grid's wavefront shadow queries on grid_stream (compact queries) against the path kernel's
#      MODE_QSTREAM over the marker layout (DRT_GRID_STREAM=0), same library, with band / wave / refill knobs
#   B: at the head with grid_stream on by default: GPU tests, smoke, the Grid PMC record, every BASELINE config
#   usage: bash tools/gstream_session.sh A|B
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
G="--accel grid"
case "${1:-A}" in
  A)
    timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/gpu_tests.log 2>&1
    rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
    STEPS=6 bash tools/lib_matrix.sh 2 "gs||$G" "qstream|DRT_GRID_STREAM=0|$G" "gs_b8|DRT_WAVEFRONT_BANDS=8|$G" \
      "gs_w6|DRT_WAVEFRONT_GRID_WAVES=6|$G" "gs_w5|DRT_WAVEFRONT_GRID_WAVES=5|$G" "gs_r8|DRT_WAVEFRONT_GRID_REFILL_MIN=8|$G" || exit $?
    cp $OUT/lib_matrix.jsonl $OUT/gstream_ab.jsonl
    ;;
  B)
    bash tools/session.sh tests smoke || exit $?
    cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
    PMC_ONLY="grid" PMC_DB=$OUT/pmc_traffic.json bash tools/pmc_configs.sh || exit $?
    CFG_STEPS=10 bash tools/configs.sh || exit $?
    ;;
  *)
    echo "unknown part $1"; exit 2 ;;
esac
