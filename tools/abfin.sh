#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; grep -E "FAILED|passed|failed" gpurun_out/gpu_tests.log | tail -3; [ $rc -ne 0 ] && exit $rc
bash tools/ab3.sh 3 "base:AVT_LIB_PATH=$(pwd)/audio-visual-tubes_amd/libavt_base.so" "new:"
BENCH_ARGS="--batch 32 --steps 20" bash tools/ab3.sh 2 "b32base:AVT_LIB_PATH=$(pwd)/audio-visual-tubes_amd/libavt_base.so" "b32new:"
