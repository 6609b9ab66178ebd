#!/bin/bash
# Rehearse bench.py's N>1 path (tile shards, all-gather, unshard, max-over-ranks timing) with
# NPROC (default 2) ranks folded onto one GPU over gloo (RCCL refuses two ranks on one device).  The real N>1
# runs use RCCL, one rank per GPU.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
N=${NPROC:-2}
DRT_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $N --steps ${STEPS:-2} --warmup 1 --res 256 --spp 16 \
  --check-frame > $OUT/mr$N.json 2> $OUT/mr$N.err
rc=$?; echo "$N-rank rc=$rc"; cut -c1-300 $OUT/mr$N.json; grep -o "\"frame_check[a-z_]*\": [a-z]*" $OUT/mr$N.json; tail -3 $OUT/mr$N.err; exit $rc
