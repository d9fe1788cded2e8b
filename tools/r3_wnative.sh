#!/bin/bash
# Round 3: TN wgrad with the register-order slab epilogue + native reduce: tests, per-shape sweep, step A/B vs HEAD
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
B=$(pwd)/audio-visual-tubes_amd/libavt_base.so
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad" > gpurun_out/t_wgrad.log 2>&1; rc=$?
echo "wgrad tests rc=$rc"; tail -3 gpurun_out/t_wgrad.log; [ $rc -ne 0 ] && exit $rc
for Bt in 32 128; do
for lib in base new; do
  if [ $lib = base ]; then export AVT_LIB_PATH=$B; else unset AVT_LIB_PATH; fi
  timeout -k 10 300 python tools/conv_bench.py --batch $Bt --kinds wgrad --variants 1 > gpurun_out/cbw.txt 2>&1 || { tail -5 gpurun_out/cbw.txt; exit 1; }
  echo "== B=$Bt $lib"; grep -v amdgpu gpurun_out/cbw.txt | sed 's/wgrad\[h0,t1,0,4,n4,3\]//g'
done; done
unset AVT_LIB_PATH
timeout -k 10 300 python tools/conv_bench.py --batch 32 --kinds wgrad --variants 1 --slab-max "32,4;32,8" > /dev/null 2>&1
for wc in 4 8 16; do
timeout -k 10 300 python tools/conv_bench.py --batch 32 --kinds wgrad --variants 1 --slab-max "32,$wc" > gpurun_out/cbw.txt 2>&1 || { tail -5 gpurun_out/cbw.txt; exit 1; }
echo "== B=32 wave_cost $wc"; grep -v amdgpu gpurun_out/cbw.txt | tail -1
done
for mk in 4 8 12; do
AVT_WGRAD_MIN_KT_1X1=$mk timeout -k 10 300 python tools/conv_bench.py --batch 32 --only "ds" --kinds wgrad --variants 1 > gpurun_out/cbw.txt 2>&1 || { tail -5 gpurun_out/cbw.txt; exit 1; }
echo "== B=32 1x1 min_kt $mk"; grep -v amdgpu gpurun_out/cbw.txt | sed 's/wgrad\[h0,t1,0,4,n4,3\]//g'
done
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 2 "base:AVT_LIB_PATH=$B" "new:" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 2 "base:AVT_LIB_PATH=$B" "new:" || exit 1
