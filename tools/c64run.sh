#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "c64 or conv_dgrad or conv_fwd or halo" > gpurun_out/k.log 2>&1; rc=$?; tail -3 gpurun_out/k.log; [ $rc -ne 0 ] && exit $rc
CB_ARGS="--only l1 --variants 1 --kinds fwd,dgrad" timeout -k 10 200 python tools/conv_bench.py --only l1 --variants 1 --kinds fwd,dgrad --halo 1 > gpurun_out/cb.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/cb.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-400; exit $rc
