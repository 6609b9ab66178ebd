#!/bin/bash
# Round-6 Grid session (f4): the indexed single-copy layout at the head, the Grid caps re-tuned at 7 waves/SIMD,
# and the chain passes' instruction mix with f64 VALU counters (headline BVH vs Grid).
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
GIDX=DRT_LIBRARY=distributionraytracer_amd/csrc/build/alt/libdrt_gidx.so
env $GIDX timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "grid" > $OUT/gidx_tests.log 2>&1
rc=$?; tail -2 $OUT/gidx_tests.log; [ $rc -eq 0 ] || exit $rc
G="--accel grid"
STEPS=5 bash tools/lib_matrix.sh 2 "grid||$G" "gidx|$GIDX|$G" "cp2|DRT_CHAIN_GRID_PAIRS=2|$G" "cp4|DRT_CHAIN_GRID_PAIRS=4|$G" \
  "cw5|DRT_CHAIN_GRID_WALK=5|$G" "qp2|DRT_REPLAY_GRID_PAIRS=2|$G" "qp4|DRT_REPLAY_GRID_PAIRS=4|$G" "qw5|DRT_REPLAY_GRID_WALK=5|$G" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/grid_knobs.jsonl
CNT="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"
for cfg in "bvh:" "grid:--accel grid"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CNT -d $OUT/pmc_f64/$name -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --settle-s 0 --no-cpu-baseline --no-load-timing $args > $OUT/pmc_f64_$name.json 2> $OUT/pmc_f64_$name.err
  rc=$?; echo "pmc f64 $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_passes.py $OUT/pmc_f64/bvh > $OUT/pmc_f64_bvh_kernels.json && python3 tools/pmc_passes.py $OUT/pmc_f64/grid > $OUT/pmc_f64_grid_kernels.json
