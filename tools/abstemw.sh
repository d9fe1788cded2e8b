#!/bin/bash
# audio stem wgrad with two tiles in flight per wave: stem tests, stem wgrad per-shape (base vs new), step A/B at B=128
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
B=$(pwd)/audio-visual-tubes_amd/libavt_base.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "stem" > gpurun_out/k.log 2>&1; rc=$?; tail -1 gpurun_out/k.log; [ $rc -ne 0 ] && { grep -E "^(FAILED|E )" gpurun_out/k.log | head -30; exit $rc; }
for i in 1 2; do AVT_LIB_PATH=$B timeout -k 10 120 python tools/stem_wgrad_bench.py 2>&1 | grep stem | sed 's/^/base /' && timeout -k 10 120 python tools/stem_wgrad_bench.py 2>&1 | grep stem | sed 's/^/new  /' || exit 1; done
bash tools/ab3.sh 3 "base:AVT_LIB_PATH=$B" "new:"
