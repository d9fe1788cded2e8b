#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad or stem" > gpurun_out/k.log 2>&1; rc=$?; tail -2 gpurun_out/k.log; [ $rc -ne 0 ] && exit $rc
for l in base new; do
  if [ $l = base ]; then E="AVT_LIB_PATH=$(pwd)/audio-visual-tubes_amd/libavt_base.so"; else E="AVT_X=1"; fi
  env $E timeout -k 10 200 python tools/conv_bench.py --variants 1 --kinds wgrad 2>&1 | grep -v amdgpu | sed "s/^/$l /"
done
bash tools/ab3.sh 3 "base:AVT_LIB_PATH=$(pwd)/audio-visual-tubes_amd/libavt_base.so" "new:"
