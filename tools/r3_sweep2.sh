#!/bin/bash
# Round 3: layer4 wgrad on the 128x128 two-group kernel vs the 256x256 tile; small halo ring depth at B=32
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
for Bt in 32 128; do
  timeout -k 10 300 python tools/conv_bench.py --batch $Bt --only "l4" --kinds wgrad --variants 1 --wgrad-tiles 1,0 > gpurun_out/cbw.txt 2>&1 || { tail -5 gpurun_out/cbw.txt; exit 1; }
  echo "== B=$Bt tiles 1,0"; grep -v amdgpu gpurun_out/cbw.txt | sed 's/wgrad\[h0,//g'
done
timeout -k 10 300 python tools/conv_bench.py --batch 32 --only "3x3" --kinds none --variants 1 --stages "2,2;2,3;2,4;2,5" > gpurun_out/cbs.txt 2>&1 || { tail -5 gpurun_out/cbs.txt; exit 1; }
echo "== B=32 small halo stages"; grep -v amdgpu gpurun_out/cbs.txt
