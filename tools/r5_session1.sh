#!/bin/bash
# Round-5 session: the two-pass plan tests (size rule), then the headline and Grid bench lines with
# per-pass roofline rows.  Stops at the first failing step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "two_pass or size_rule" --timeout 300 --timeout-method thread > $OUT/t_plan.log 2>&1
rc=$?; tail -n 3 $OUT/t_plan.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_head.json 2> $OUT/bench_head.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-load-timing --accel grid > $OUT/bench_grid.json 2> $OUT/bench_grid.err
rc=$?; echo "bench grid rc=$rc"; [ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json
for f in ("gpurun_out/bench_head.json", "gpurun_out/bench_grid.json"):
    d = json.load(open(f)); r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], r["frac"], r.get("frac_ref_tree"), r.get("pass_sum_ms"), r["kernel_ms_serial"])
    for p in r.get("passes") or []: print("  ", p)
PY
