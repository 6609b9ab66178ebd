#!/bin/bash
# Round-5: per-rank shard frame times (tools/shard_scaling.py) with the wavefront replay, frames in
# flight 1 / 2 / 3.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
for p in 1 2 3; do
  timeout -k 10 400 python tools/shard_scaling.py --steps 40 --pipe $p > $OUT/shard_pipe$p.json 2> $OUT/shard_pipe$p.err || exit $?
  tail -c 600 $OUT/shard_pipe$p.json; echo
done
