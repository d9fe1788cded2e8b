#!/bin/bash
# Round 3: split-K head GEMMs at short grids: head tests, step A/B vs HEAD
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
B=$(pwd)/audio-visual-tubes_amd/libavt_base.so
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_boundary_gpu.py tests/test_twoview_gpu.py tests/test_tube_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "hardway or model or boundary or twoview or tube or head" > gpurun_out/t_head.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/t_head.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 3 "base:AVT_LIB_PATH=$B" "new:" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 2 "base:AVT_LIB_PATH=$B" "new:" || exit 1
