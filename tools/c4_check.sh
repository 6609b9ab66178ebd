set -u
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
bash tools/ab.sh "DRT_WAVES=6" || exit $?
C4="--res 1024 --spp 64 --aperture 8 --focal 1 --max-depth 8 --roughness 0.1 --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python bench.py $C4 > $OUT/c4_persistent.json 2> $OUT/c4_persistent.err || exit $?
cut -c1-400 $OUT/c4_persistent.json
DRT_PERSISTENT=0 timeout -k 10 400 python bench.py $C4 --steps 1 --warmup 0 > $OUT/c4_megakernel.json 2> $OUT/c4_megakernel.err || exit $?
cut -c1-400 $OUT/c4_megakernel.json
