#!/bin/bash
# Round-end evidence in one GPU session: PMC passes of the timed path kernel (HBM traffic per
# launch -> profiles/pmc_traffic.json, read by bench.py), then tests / smoke / bench / rocprof
# stats (tools/gpu_check.sh).  Outputs land in gpurun_out/ (copy the ones to keep into profiles/).
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
STEPS=1 bash tools/pmc.sh "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
  "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE" \
  "TCP_TOTAL_CACHE_ACCESSES TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY" || exit $?
python tools/pmc_traffic.py $OUT/pmc tris1000000_res512_spp64 profiles/pmc_traffic.json || exit $?
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
python tools/pmc_dump.py $OUT/pmc > $OUT/pmc_dump.json || exit $?
bash tools/gpu_check.sh
