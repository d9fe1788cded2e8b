#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "c64" > gpurun_out/k.log 2>&1; rc=$?; tail -1 gpurun_out/k.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab3.sh 3 "base:AVT_LIB_PATH=$(pwd)/audio-visual-tubes_amd/libavt_base.so" "new:"
BENCH_ARGS="--batch 32 --steps 20" bash tools/ab3.sh 2 "b32base:AVT_LIB_PATH=$(pwd)/audio-visual-tubes_amd/libavt_base.so" "b32new:"
