#!/bin/bash
# Round 3: halo kernels with precomputed patch offsets (libavt.so) vs HEAD (libavt_base.so): halo tests,
# per-shape microbench, B=128 and B=32 step A/B.
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
B=$(pwd)/audio-visual-tubes_amd/libavt_base.so
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_twoview_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k "halo or conv_fwd or conv_dgrad or loss_module" > gpurun_out/t_halo.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/t_halo.log; [ $rc -ne 0 ] && exit $rc
for lib in base new; do
  if [ $lib = base ]; then export AVT_LIB_PATH=$B; else unset AVT_LIB_PATH; fi
  echo "== $lib"; timeout -k 10 300 python tools/conv_bench.py --batch 128 --only "3x3" --kinds fwd,dgrad --variants 1 2>&1 | grep -v "^{\|amdgpu" || exit 1
done
unset AVT_LIB_PATH
BENCH_ARGS="--steps 20" bash tools/ab3.sh 3 "base:AVT_LIB_PATH=$B" "new:" || exit 1
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 2 "base:AVT_LIB_PATH=$B" "new:" || exit 1
