#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "halo or conv_dgrad or conv_fwd or c64 or variants or epilogue" > gpurun_out/k.log 2>&1; rc=$?; tail -2 gpurun_out/k.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab3.sh 3 "halo1:AVT_HALO=1" "tapl2:AVT_HALO=1 AVT_HALO_L2=0"
BENCH_ARGS="--batch 32 --steps 20" bash tools/ab3.sh 2 "b32:"
