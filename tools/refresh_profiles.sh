#!/bin/bash
# Round-end evidence in two GPU sessions (outputs in gpurun_out/; copy the ones to keep into
# profiles/ under the round's prefix):
#   part A: the vector-memory gather ceilings (tools/ceiling.py -> gather_ceiling.json) and the
#           PMC records of every BASELINE config's timed path kernel (tools/pmc_configs.sh ->
#           pmc_traffic.json), both read by bench.py
#   part B: every BASELINE config (tools/configs.sh), parity tests, smoke, bench, and a rocprofv3
#           --kernel-trace --stats run of the same bench command whose path-kernel time per step
#           (tools/rocprof_union.py) bench's HIP events must match
#   usage: bash tools/refresh_profiles.sh A|B
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
case "${1:-A}" in
  A)
    timeout -k 10 300 python tools/ceiling.py $OUT/gather_ceiling.json || exit $?
    cp $OUT/gather_ceiling.json profiles/gather_ceiling.json
    PMC_DB=$OUT/pmc_traffic.json bash tools/pmc_configs.sh || exit $?
    ;;
  B)
    bash tools/configs.sh || exit $?
    STEPS=${STEPS:-10} bash tools/gpu_check.sh || exit $?
    ;;
esac
