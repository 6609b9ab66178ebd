#!/bin/bash
# One GPU session as a list of steps, run in order; the session stops at the first step that fails,
# faults or times out (every GPU step runs under its own timeout).  Replaces the one-shot
# r4_session*/r5_session* scripts of rounds 4-5.
#
#   bash tools/session.sh STEP [STEP ...]
#
# Steps:
#   tests[:EXPR]          pytest -m gpu over tests/ (-k EXPR if given)        -> gpurun_out/gpu_tests.log
#   smoke                 __graft_entry__.smoke()                              -> gpurun_out/smoke.log
#   bench[:ARGS]          python bench.py ARGS (default: the headline, 10 steps)  -> gpurun_out/bench.json
#   prof[:ARGS]           rocprofv3 --kernel-trace --stats of bench.py ARGS + tools/rocprof_union.py
#   mr:N                  tools/multirank_check.sh with N gloo ranks on the one GPU  -> gpurun_out/mrN.json
#   matrix:REPS:S1;S2;..  tools/lib_matrix.sh REPS S1 S2 ... (S = "label|ENV=..|bench args")
#                                                                     -> gpurun_out/matrix_<k>.jsonl
#   configs               tools/configs.sh (every BASELINE config with its CPU baseline)
#   shards:ARGS           tools/shard_scaling.py ARGS                         -> gpurun_out/shards_<k>.json
#   pmc:NAMES             tools/pmc_configs.sh for the named configs ("headline c3 grid c4 c2")
set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
k=0
for step in "$@"; do
  k=$((k + 1))
  name=${step%%:*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*:}
  echo "== step $k: $step"
  case $name in
    tests)
      if [ -n "$arg" ]; then
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$arg" \
          > $OUT/gpu_tests.log 2>&1
      else
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
          > $OUT/gpu_tests.log 2>&1
      fi
      rc=$?; tail -3 $OUT/gpu_tests.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; tail -2 $OUT/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py ${arg:---steps 10 --warmup 2} > $OUT/bench.json 2> $OUT/bench.err
      rc=$?; cut -c1-400 $OUT/bench.json; tail -2 $OUT/bench.err ;;
    prof)
      a=${arg:---steps 10 --warmup 2}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
        python3 bench.py $a --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err
      rc=$?
      if [ $rc -eq 0 ]; then
        st=$(echo "$a" | sed -n 's/.*--steps \([0-9]*\).*/\1/p'); wu=$(echo "$a" | sed -n 's/.*--warmup \([0-9]*\).*/\1/p')
        python tools/rocprof_union.py $OUT/prof --steps ${st:-10} --warmup ${wu:-2} --bench-json $OUT/prof_bench.json \
          > $OUT/rocprof_union.json
        rc=$?; cut -c1-400 $OUT/rocprof_union.json
      fi ;;
    mr)
      NPROC=$arg bash tools/multirank_check.sh; rc=$? ;;
    matrix)
      reps=${arg%%:*}; specs=${arg#*:}
      IFS=';' read -r -a S <<< "$specs"
      bash tools/lib_matrix.sh $reps "${S[@]}"; rc=$?
      cp $OUT/lib_matrix.jsonl $OUT/matrix_$k.jsonl 2>/dev/null ;;
    configs)
      bash tools/configs.sh; rc=$? ;;
    shards)
      timeout -k 10 900 python tools/shard_scaling.py $arg > $OUT/shards_$k.json 2> $OUT/shards_$k.err
      rc=$?; tail -c 600 $OUT/shards_$k.json ;;
    pmc)
      PMC_ONLY="$arg" bash tools/pmc_configs.sh; rc=$? ;;
    *)
      echo "unknown step $name"; rc=2 ;;
  esac
  echo "== step $k rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
