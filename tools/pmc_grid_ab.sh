#!/bin/bash
# PMC passes of the Grid headline kernel for two library builds (fabric lines, hit rates, load
# instructions): A = the default build, B = $B_LIB.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmc_grid; mkdir -p $OUT
GROUPS_=("TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum"
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
  "TA_TA_BUSY TD_TD_BUSY TCP_TOTAL_CACHE_ACCESSES GRBM_GUI_ACTIVE" "WRITE_SIZE")
for v in A B; do
  i=0; mkdir -p $OUT/$v
  for grp in "${GROUPS_[@]}"; do
    i=$((i+1))
    if [ $v = B ]; then E="DRT_LIBRARY=$B_LIB"; else E="DRT_NONE=1"; fi
    env $E timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d $OUT/$v/p$i -o run --output-format csv -- \
        python3 bench.py --steps 1 --warmup 0 --settle-s 0 --no-cpu-baseline --no-load-timing --accel grid \
        > $OUT/$v/p$i.json 2> $OUT/$v/p$i.err
    rc=$?; echo "$v pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 - <<'PY'
import csv, json
from pathlib import Path
res = {}
for v in ("A", "B"):
    tot = {}
    for f in Path(f"gpurun_out/pmc_grid/{v}").rglob("*counter_collection.csv"):
        rows = list(csv.DictReader(open(f)))
        disp = {}
        for r in rows:
            if "path_persistent" in r["Kernel_Name"] and ", false," in r["Kernel_Name"]:
                disp.setdefault(int(r["Dispatch_Id"]), {}).setdefault(r["Counter_Name"], 0.0)
                disp[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        if disp:
            last = disp[max(disp)]
            tot.update(last)
    res[v] = tot
print(json.dumps(res, indent=1))
json.dump(res, open("gpurun_out/pmc_grid/summary.json", "w"), indent=1)
PY
