#!/bin/bash
# Round 3: BN finalize folded into the apply launch (AVT_BN_FIN): kernel + model tests, step A/B
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_boundary_gpu.py tests/test_schedule_gpu.py tests/test_fullsize_gpu.py tests/test_twoview_gpu.py tests/test_tube_gpu.py tests/test_splitk_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_fin.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/t_fin.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 3 "fin0:AVT_BN_FIN=0" "fin1:" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 2 "fin0:AVT_BN_FIN=0" "fin1:" || exit 1
