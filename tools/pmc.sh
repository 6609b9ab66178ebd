#!/bin/bash
# PMC passes over the bench (one rocprofv3 run per counter group, kernel trace only).
set -u
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}; mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- \
      python3 bench.py --steps ${STEPS:-1} --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/p$i.json 2> $OUT/p$i.err
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
