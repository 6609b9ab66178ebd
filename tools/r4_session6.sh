#!/bin/bash
# Knob re-check at the round-4 head (replay / chain batch sizes on the headline, C3 and the Grid) and
# the 8-way shard with four frames in flight.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
C3="--tris 100000 --light-spp 4"; G="--accel grid"
bash tools/lib_matrix.sh 1 "head|DRT_X=1|" "rpm16|DRT_REPLAY_PROCESS_MIN=16|" "rpm20|DRT_REPLAY_PROCESS_MIN=20|" "rpm32|DRT_REPLAY_PROCESS_MIN=32|" \
  "rrf4|DRT_REPLAY_REFILL_MIN=4|" "rrf12|DRT_REPLAY_REFILL_MIN=12|" "head2|DRT_X=1|" \
  "c3|DRT_X=1|$C3" "c3_rpm16|DRT_REPLAY_PROCESS_MIN=16|$C3" "c3_rpm32|DRT_REPLAY_PROCESS_MIN=32|$C3" \
  "grid|DRT_X=1|$G" "grid_rpm16|DRT_REPLAY_PROCESS_MIN=16|$G" "grid_rpm32|DRT_REPLAY_PROCESS_MIN=32|$G" "grid_cpm16|DRT_CHAIN_PROCESS_MIN=16|$G" || exit $?
cp $OUT/lib_matrix.jsonl $OUT/knobs6.jsonl
timeout -k 10 300 python tools/shard_scaling.py --pipe 4 --steps 40 --shards 8 > $OUT/shard_p4.json 2> $OUT/shard_p4.err
rc=$?; tail -n 1 $OUT/shard_p4.json | cut -c1-400; exit $rc
