#!/bin/bash
# Round-5 evidence at the head: GPU suite, smoke, every BASELINE config (10 steps), the bench line and a
# rocprofv3 kernel trace of the same command, Whitted one- vs two-pass frames on the shipped scenes, and
# the multi-GPU projection (per-rank shard time, three frames in flight, 40 steps).  Stops at the first
# failing step.
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -n 3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -n 1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
CFG_STEPS=10 bash tools/configs.sh || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/rocprof_union.py $OUT/prof --steps 20 --warmup 5 --bench-json $OUT/prof_bench.json > $OUT/rocprof_union.json || exit $?
cat $OUT/rocprof_union.json
timeout -k 10 300 python tools/whitted_two_pass.py --frames 20 > $OUT/whitted_two_pass.jsonl 2> $OUT/whitted_two_pass.err
rc=$?; echo "whitted rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/shard_scaling.py --pipe 3 --steps 40 --shards 1,2,4,8 > $OUT/shard_scaling.json 2> $OUT/shard_scaling.err
rc=$?; echo "shard rc=$rc"; tail -2 $OUT/shard_scaling.json | cut -c1-300; exit $rc
