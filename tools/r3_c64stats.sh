#!/bin/bash
# Round 3: c64 BN partials per block (one set of atomics per block, not per tile): tests, step A/B vs
# HEAD (libavt_base.so), then the two-stream finalize probe
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
B=$(pwd)/audio-visual-tubes_amd/libavt_base.so
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "c64 or conv or model or hardway or bn" > gpurun_out/t_c64.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/t_c64.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 2 "base:AVT_LIB_PATH=$B" "new:" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 2 "base:AVT_LIB_PATH=$B" "new:" || exit 1
bash tools/r3_finprobe.sh
