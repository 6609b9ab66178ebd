#!/bin/bash
# Rehearse bench.py's N>1 path (tile shards, all-gather, unshard, max-over-ranks timing) with
# 2 ranks folded onto one GPU over gloo (RCCL refuses two ranks on one device).  The real N>1
# runs use RCCL, one rank per GPU.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
DRT_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 --res 256 --spp 16 --check-frame \
  > $OUT/mr2.json 2> $OUT/mr2.err
rc=$?; echo "2-rank rc=$rc"; cut -c1-300 $OUT/mr2.json; grep -o "\"frame_check[a-z_]*\": [a-z]*" $OUT/mr2.json; tail -3 $OUT/mr2.err; exit $rc
