#!/bin/bash
# PMC passes of the timed path-kernel dispatch for every BASELINE config on one GPU (headline, C3,
# C4, the headline scene on the Grid, C2), one rocprofv3 run per counter group, merged per workload key
# into profiles/pmc_traffic.json (tools/pmc_traffic.py; bench.py reads its key's record).
set -u
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc_cfg}; mkdir -p $OUT
DB=${PMC_DB:-$OUT/pmc_traffic.json}
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
  "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
  "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE"
  "TCP_TOTAL_CACHE_ACCESSES TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY")
CONFIGS=("headline:" "c3:--tris 100000 --light-spp 4" "grid:--accel grid"
  "c4:--res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8" "c2:--scene balls_low --spp 16")
for cfg in "${CONFIGS[@]}"; do
  name=${cfg%%:*}; args=${cfg#*:}
  # PMC_ONLY="c2 grid": only those configs (their records are merged into the existing database)
  if [ -n "${PMC_ONLY:-}" ] && [[ " $PMC_ONLY " != *" $name "* ]]; then continue; fi
  mkdir -p $OUT/$name
  i=0
  for grp in "${GROUPS_[@]}"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d $OUT/$name/p$i -o run --output-format csv -- \
        python3 bench.py --steps 1 --warmup 0 --settle-s 0 --no-cpu-baseline $args > $OUT/$name/p$i.json 2> $OUT/$name/p$i.err
    rc=$?; echo "$name pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  key=$(python3 -c "import json;print(json.load(open('$OUT/$name/p1.json'))['config']['key'])")
  python3 tools/pmc_traffic.py $OUT/$name $key $DB || exit $?
done
