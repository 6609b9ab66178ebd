#!/bin/bash
# Round-end evidence at the head, in two GPU calls (outputs in gpurun_out/):
#   X: parity tests, smoke, the gather ceilings (tools/ceiling.py) and the PMC records of the headline, C3 and
#      Grid configs (tools/pmc_configs.sh)
#   Y: the PMC records of C4 and C2, every BASELINE config (tools/configs.sh, 10 steps, CPU baselines), the
#      bench line and a rocprofv3 --kernel-trace --stats run of the same command (tools/gpu_check.sh, no tests)
#   Z: Y without the PMC passes, plus the 2-rank multi-rank rehearsal (tools/multirank_check.sh)
#   G: the Grid PMC record after grid_stream + Z's bench evidence; H: tests, smoke, multi-rank, shard scaling
#   F: the Grid PMC record after the Grid shadow tree, tests, smoke, configs, bench + rocprof union
#   usage: bash tools/final_session.sh X|Y|Z|G|H|F
set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
case "${1:-X}" in
  X)
    bash tools/session.sh tests smoke || exit $?
    timeout -k 10 300 python tools/ceiling.py $OUT/gather_ceiling.json || exit $?
    PMC_ONLY="headline c3 grid" PMC_DB=$OUT/pmc_traffic.json bash tools/pmc_configs.sh || exit $?
    ;;
  Y)
    PMC_ONLY="c4 c2" PMC_DB=$OUT/pmc_traffic.json bash tools/pmc_configs.sh || exit $?
    CFG_STEPS=10 bash tools/configs.sh || exit $?
    timeout -k 10 600 python bench.py --steps 20 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || exit $?
    cut -c1-300 $OUT/bench.json
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
        python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || exit $?
    python tools/rocprof_union.py $OUT/prof --steps 20 --warmup 2 --bench-json $OUT/prof_bench.json > $OUT/rocprof_union.json || exit $?
    cat $OUT/rocprof_union.json
    ;;
  Z)  # the head's bench evidence after a change that needs no new PMC records: Y without its PMC passes, plus
      # the multi-rank rehearsal
    CFG_STEPS=10 bash tools/configs.sh || exit $?
    timeout -k 10 600 python bench.py --steps 20 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || exit $?
    cut -c1-300 $OUT/bench.json
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
        python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || exit $?
    python tools/rocprof_union.py $OUT/prof --steps 20 --warmup 2 --bench-json $OUT/prof_bench.json > $OUT/rocprof_union.json || exit $?
    cat $OUT/rocprof_union.json
    NPROC=2 bash tools/multirank_check.sh || exit $?
    ;;
  G)  # after grid_stream: the Grid's PMC record (its pass-2 stream now counted), then Z's bench evidence with
      # that record in the database the bench reads
    cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
    PMC_ONLY="grid" PMC_DB=$OUT/pmc_traffic.json bash tools/pmc_configs.sh || exit $?
    cp $OUT/pmc_traffic.json profiles/pmc_traffic.json
    CFG_STEPS=10 bash tools/configs.sh || exit $?
    timeout -k 10 600 python bench.py --steps 20 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || exit $?
    cut -c1-300 $OUT/bench.json
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
        python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || exit $?
    python tools/rocprof_union.py $OUT/prof --steps 20 --warmup 2 --bench-json $OUT/prof_bench.json > $OUT/rocprof_union.json || exit $?
    cat $OUT/rocprof_union.json
    ;;
  F)  # after the Grid scene's shadow tree: the Grid PMC record (its pass 2 now trace_stream GV + grid_stream),
      # the parity tests, smoke, every config, the bench line and its rocprof union
    cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
    PMC_DB=$OUT/pmc_traffic.json bash tools/session.sh "pmc:grid" || exit $?
    cp $OUT/pmc_traffic.json profiles/pmc_traffic.json
    CFG_STEPS=10 bash tools/session.sh tests smoke configs "bench:--steps 20 --warmup 2" "prof:--steps 20 --warmup 2" || exit $?
    ;;
  H)  # the parity tests, smoke, the multi-rank rehearsal and the shard scaling at the head
    bash tools/session.sh tests smoke mr:2 "shards:--steps 40 --pipe 2" || exit $?
    ;;
  *)
    echo "unknown part $1"; exit 2 ;;
esac
