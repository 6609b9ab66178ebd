set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "two_pass or grid" --timeout 300 --timeout-method thread > gpurun_out/t_grid2p.log 2>&1
rc=$?; tail -n 5 gpurun_out/t_grid2p.log; [ $rc -eq 0 ] || exit $rc
P=distributionraytracer_amd/csrc/build/alt/libdrt_prev.so
K=distributionraytracer_amd/csrc/build/alt/libdrt_wpk.so
bash tools/lib_matrix.sh 2 "o0|DRT_WIDE_ORDER=0|" "o2|DRT_WIDE_ORDER=2|" "prev_o0|DRT_LIBRARY=$P DRT_WIDE_ORDER=0|" "prev_o1|DRT_LIBRARY=$P DRT_WIDE_ORDER=1|" "prev_o2|DRT_LIBRARY=$P DRT_WIDE_ORDER=2|" "wpk_o2|DRT_LIBRARY=$K DRT_WIDE_ORDER=2|" "grid|DRT_X=1|--accel grid" "grid_cpm16|DRT_CHAIN_PROCESS_MIN=16|--accel grid" "grid_cpm24|DRT_CHAIN_PROCESS_MIN=24|--accel grid" "grid_cpm4|DRT_CHAIN_PROCESS_MIN=4|--accel grid"
