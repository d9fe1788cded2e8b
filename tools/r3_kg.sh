#!/bin/bash
# Round 3: two wave groups per TN wgrad block (AVT_WGRAD_KG): tests, per-shape, step A/B
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad" > gpurun_out/t_wgrad.log 2>&1; rc=$?
echo "wgrad tests rc=$rc"; tail -2 gpurun_out/t_wgrad.log; [ $rc -ne 0 ] && exit $rc
for Bt in 32 128; do for kg in 1 2; do
  AVT_WGRAD_KG=$kg timeout -k 10 300 python tools/conv_bench.py --batch $Bt --kinds wgrad --variants 1 > gpurun_out/cbw.txt 2>&1 || { tail -5 gpurun_out/cbw.txt; exit 1; }
  echo "== B=$Bt kg=$kg"; grep -v amdgpu gpurun_out/cbw.txt | sed 's/wgrad\[h0,t1,0,4,n4,3\]//g'
done; done
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 3 "kg1:AVT_WGRAD_KG=1" "kg2:" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 2 "kg1:AVT_WGRAD_KG=1" "kg2:" || exit 1
