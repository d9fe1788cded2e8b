#!/bin/bash
# Round 3: BN statistic slots 64 vs 16 (libavt_base.so = working tree with -DAVT_BN_SLOTS=16); BN finalize
# in the apply launch on top (AVT_BN_FIN): BN/model tests, step A/B
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
B=$(pwd)/audio-visual-tubes_amd/libavt_base.so
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_boundary_gpu.py tests/test_fullsize_gpu.py tests/test_tube_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_slots.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/t_slots.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 2 "s16:AVT_LIB_PATH=$B AVT_BN_FIN=0" "s64:AVT_BN_FIN=0" "s64fin:" "s64skip:AVT_BN_FIN=0 AVT_DIAG_SKIP=1" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 2 "s16:AVT_LIB_PATH=$B AVT_BN_FIN=0" "s64:AVT_BN_FIN=0" "s64fin:" "s64skip:AVT_BN_FIN=0 AVT_DIAG_SKIP=1" || exit 1
