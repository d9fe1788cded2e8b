#!/bin/bash
# Round 3: 16-lane BN finalize kernels + TN register-order slab; nst_big A/B; tests
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
B=$(pwd)/audio-visual-tubes_amd/libavt_base.so
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_fin.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/t_fin.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 3 "base:AVT_LIB_PATH=$B" "new:" "nb4:AVT_WGRAD_NST_BIG=4" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 3 "base:AVT_LIB_PATH=$B" "new:" "nb4:AVT_WGRAD_NST_BIG=4" || exit 1
