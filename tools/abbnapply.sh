#!/bin/bash
# bn_apply with two vectors in flight per thread: BN tests, step A/B against the HEAD build (B=128, B=32)
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
B=$(pwd)/audio-visual-tubes_amd/libavt_base.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "bn or model or step" > gpurun_out/k.log 2>&1; rc=$?; tail -1 gpurun_out/k.log; [ $rc -ne 0 ] && { grep -E "^(FAILED|E )" gpurun_out/k.log | head -30; exit $rc; }
bash tools/ab3.sh 3 "base:AVT_LIB_PATH=$B" "new:" && BENCH_ARGS="--batch 32 --steps 20" bash tools/ab3.sh 2 "base32:AVT_LIB_PATH=$B" "new32:"
