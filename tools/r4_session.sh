#!/bin/bash
# Round-4 evidence session: GPU tests, smoke, bench, streaming shadow kernel on both trees,
# rocprofv3 of the bench.  Stops at the first failing step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/gpu_tests.log
if [ $rc -ge 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
for flag in "" "--reference-order"; do
  timeout -k 10 300 python tools/trace_bench.py --waves 6,8 --reps 3 $flag > $OUT/trace_bench$flag.log 2>&1
  rc=$?; echo "trace_bench $flag rc=$rc"; grep -E "^shadow" $OUT/trace_bench$flag.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python bench.py --steps ${STEPS:-20} --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
