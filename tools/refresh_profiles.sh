#!/bin/bash
# Round-end evidence in one GPU session (outputs in gpurun_out/; copy the ones to keep into
# profiles/ under the round's prefix):
#   1. the vector-memory gather ceiling (tools/ceiling.py -> gather_ceiling.json, read by bench.py)
#   2. PMC passes of the timed path kernel: HBM traffic per launch (-> pmc_traffic.json, read by
#      bench.py) and the pipe counters
#   3. parity tests, smoke, bench, and a rocprofv3 --kernel-trace --stats run of the same bench
#      command whose path-kernel time per step (tools/rocprof_union.py) bench's HIP events must match
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python tools/ceiling.py $OUT/gather_ceiling.json || exit $?
cp $OUT/gather_ceiling.json profiles/gather_ceiling.json
STEPS=1 bash tools/pmc.sh "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
  "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE" \
  "TCP_TOTAL_CACHE_ACCESSES TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY" \
  "SQ_INSTS_VMEM_WR SQ_INSTS_FLAT TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" || exit $?
python tools/pmc_traffic.py $OUT/pmc tris1000000_res512_spp64 profiles/pmc_traffic.json || exit $?
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
python tools/pmc_dump.py $OUT/pmc > $OUT/pmc_dump.json || exit $?
STEPS=${STEPS:-10} bash tools/gpu_check.sh || exit $?
