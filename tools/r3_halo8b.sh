#!/bin/bash
# Round 3: layer3/4 8-wave halo tile rule (AVT_HALO8): kernel tests, per-shape rates, step A/B
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "conv or halo or model or hardway" > gpurun_out/t_h8.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/t_h8.log; [ $rc -ne 0 ] && exit $rc
for h in 0 1; do
AVT_HALO8=$h timeout -k 10 300 python tools/conv_bench.py --batch 128 --only "3x3" --kinds none --variants 1 > gpurun_out/cbh.txt 2>&1 || { tail -5 gpurun_out/cbh.txt; exit 1; }
echo "== B=128 AVT_HALO8=$h"; grep -E "l3|l4" gpurun_out/cbh.txt
done
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 3 "h8=0:AVT_HALO8=0" "h8=1:" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 3 "h8=0:AVT_HALO8=0" "h8=1:" || exit 1
