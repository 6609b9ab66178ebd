#!/bin/bash
# Counter reset of both passes before the first (no fill kernel between the passes): two-pass parity
# tests, bench A/B against the previous build, and the 8-way shard projection.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "two_pass or slot or sharded" --timeout 300 --timeout-method thread > $OUT/t_ctr.log 2>&1
rc=$?; tail -n 2 $OUT/t_ctr.log; [ $rc -eq 0 ] || exit $rc
bash tools/lib_matrix.sh 2 "head|DRT_X=1|" "prev|DRT_LIBRARY=distributionraytracer_amd/csrc/build/alt/libdrt_prevctr.so|" || exit $?
timeout -k 10 400 python tools/shard_scaling.py --pipe 3 --steps 40 --shards 1,8 > $OUT/shard_ctr.json 2> $OUT/shard_ctr.err
rc=$?; tail -n 1 $OUT/shard_ctr.json | cut -c1-500; exit $rc
