#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprofv3 kernel trace of the same bench
# command.  Stops at the first step that faults, aborts or times out (exit >= 2 from pytest, any
# non-zero from the others).
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
S=${STEPS:-10}; W=${WARMUP:-2}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/gpu_tests.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps $S --warmup $W > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err; [ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
      python3 bench.py --steps $S --warmup $W --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err
  rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python tools/rocprof_union.py $OUT/prof --steps $S --warmup $W --bench-json $OUT/prof_bench.json > $OUT/rocprof_union.json || exit $?
  cat $OUT/rocprof_union.json
fi
