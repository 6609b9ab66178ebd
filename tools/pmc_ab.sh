#!/bin/bash
# PMC counters of the timed path-kernel dispatch for several libdrt builds (A/B), one rocprofv3
# pass per (build, counter group).  Usage:
#   LIBS="base build/alt/libdrt_x.so" bash tools/pmc_ab.sh "WRITE_SIZE" "SQ_INSTS_VMEM_WR ..."
# ("base" = the in-tree libdrt.so; BENCH_ARGS adds bench.py flags).  Prints one JSON line per build.
set -u
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc_ab}; mkdir -p $OUT
li=0
for lib in ${LIBS:-base}; do
  li=$((li+1)); i=0
  for grp in "$@"; do
    i=$((i+1))
    d=$OUT/l${li}_p$i; rm -rf $d
    if [ "$lib" = base ]; then unset DRT_LIBRARY; else export DRT_LIBRARY=$PWD/$lib; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $d -o run --output-format csv -- \
        python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > $d.json 2> $d.err
    rc=$?; [ $rc -eq 0 ] || { echo "pass $lib ($grp) rc=$rc"; tail -5 $d.err; exit $rc; }
  done
  unset DRT_LIBRARY
  python3 tools/pmc_dispatch.py "$lib" $OUT/l${li}_p* || exit $?
done
