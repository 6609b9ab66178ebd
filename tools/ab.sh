#!/bin/bash
# A/B bench variants in one GPU session (no cpu baseline). Usage: bash tools/ab.sh "ENV1" "ENV2" ...
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log
if [ $rc -ge 2 ]; then exit $rc; fi
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > $OUT/ab_$i.json 2> $OUT/ab_$i.err
  rc=$?
  python - "$v" $OUT/ab_$i.json <<'PY'
import json,sys
try:
    d=json.load(open(sys.argv[2])); print(f"{sys.argv[1]:40s} {d['value']:8.1f} Mrays/s {d['ms_per_step']:8.1f} ms  simd={d['simd_eff']} cyc={d.get('cycle_share')} frac={d['roofline']['frac']}")
except Exception as e: print(sys.argv[1], 'FAILED', e)
PY
  [ $rc -eq 0 ] || exit $rc
done
