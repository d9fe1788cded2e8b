#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
for l in base new; do
  if [ $l = base ]; then E="AVT_LIB_PATH=$(pwd)/audio-visual-tubes_amd/libavt_base.so"; else E=""; fi
  env $E timeout -k 10 200 python tools/conv_bench.py --variants 1 --kinds fwd,dgrad --only "l3" 2>&1 | grep -v amdgpu | sed "s/^/$l /"
  env $E timeout -k 10 200 python tools/conv_bench.py --variants 1 --kinds fwd,dgrad --only "l4" 2>&1 | grep -v amdgpu | sed "s/^/$l /"
done
bash tools/ab3.sh 3 "base:AVT_LIB_PATH=$(pwd)/audio-visual-tubes_amd/libavt_base.so" "new:"
