#!/bin/bash
# Round 3: per-trunk packing + per-branch Adam (world 1): tests and step A/B vs HEAD
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
B=$(pwd)/audio-visual-tubes_amd/libavt_base.so
timeout -k 10 600 python -u -m pytest tests/test_schedule_gpu.py tests/test_ddp_gpu.py tests/test_model_gpu.py tests/test_boundary_gpu.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_sched.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|max \|dparam|Error" gpurun_out/t_sched.log | tail -8; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 3 "base:AVT_LIB_PATH=$B AVT_SPLIT_PACK=0 AVT_ADAM_BRANCH=0" "new:" "pack:AVT_ADAM_BRANCH=0" "adam:AVT_SPLIT_PACK=0" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 2 "base:AVT_LIB_PATH=$B AVT_SPLIT_PACK=0 AVT_ADAM_BRANCH=0" "new:" || exit 1
