#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "halo or conv_dgrad or conv_fwd or c64 or variants" > gpurun_out/k.log 2>&1; rc=$?; tail -2 gpurun_out/k.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/conv_bench.py --variants 1 --kinds fwd,dgrad > gpurun_out/cb.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/cb.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab3.sh 2 "new:" 
