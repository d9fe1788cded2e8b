#!/bin/bash
# Round 3: gan split tests/A-B, then layer3/4 halo as the 8-wave 256-row form (AVT_HALO=2) vs 4-wave 128x128
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/r3_head.sh || exit 1
for Bt in 128 32; do
timeout -k 10 300 python tools/conv_bench.py --batch $Bt --only "3x3" --kinds none --variants 1 --halo "1,2" > gpurun_out/cbh.txt 2>&1 || { tail -5 gpurun_out/cbh.txt; exit 1; }
echo "== B=$Bt halo 1,2"; grep -v amdgpu gpurun_out/cbh.txt
done
