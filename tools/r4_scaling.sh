#!/bin/bash
# Multi-GPU projection at the round-4 head: per-rank shard time of 1/2/4/8-way tile shards on one
# GPU (three frames in flight, 40 steps), AA frames in two passes (default) and in one pass.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
for v in 1 0; do
  DRT_AA_TWO_PASS=$v timeout -k 10 400 python tools/shard_scaling.py --pipe 3 --steps 40 --shards 1,2,4,8 \
    > $OUT/shard_scaling_2p$v.json 2> $OUT/shard_scaling_2p$v.err
  rc=$?; echo "two_pass=$v rc=$rc"; tail -3 $OUT/shard_scaling_2p$v.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
