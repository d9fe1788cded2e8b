#!/bin/bash
# Round 3: deep-ring TN wgrad (avt_set_wgrad_nst): tests, per-shape sweep at B=32 / B=128
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad" > gpurun_out/t_wgrad.log 2>&1; rc=$?
echo "wgrad tests rc=$rc"; tail -3 gpurun_out/t_wgrad.log; [ $rc -ne 0 ] && exit $rc
for B in 32 128; do
timeout -k 10 400 python tools/conv_bench.py --batch $B --kinds wgrad --variants 1 --wgrad-nst "4,3;6,3;8,3;8,4;8,5" > gpurun_out/cbw.txt 2>&1 || { tail -5 gpurun_out/cbw.txt; exit 1; }
echo "== B=$B"; grep -v amdgpu gpurun_out/cbw.txt | sed 's/wgrad\[h0,t1,0,4,n/[/g'
done
