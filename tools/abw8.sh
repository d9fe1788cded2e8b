#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
AVT_C64_WAVES=8 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "c64 or conv_dgrad or conv_fwd" > gpurun_out/k.log 2>&1; rc=$?; tail -1 gpurun_out/k.log; [ $rc -ne 0 ] && exit $rc
for w in 4 8; do AVT_C64_WAVES=$w timeout -k 10 200 python tools/conv_bench.py --only l1 --variants 1 --kinds fwd,dgrad 2>&1 | grep -v amdgpu | sed "s/^/w$w /" | head -2; done
bash tools/ab3.sh 3 "w4:AVT_C64_WAVES=4" "w8:AVT_C64_WAVES=8"
