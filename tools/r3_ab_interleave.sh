#!/bin/bash
# Round 3: interleaved two-stream issue.  Model tests, A/B at B=32 and B=128, then a B=32 kernel trace.
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_ddp_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/t_model.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/t_model.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 3 "il0:AVT_INTERLEAVE=0" "il1:AVT_INTERLEAVE=1" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 2 "il0:AVT_INTERLEAVE=0" "il1:AVT_INTERLEAVE=1" || exit 1
rm -rf gpurun_out/prof32
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof32" -o run -- python "$R/bench.py" --batch 32 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof32.log 2>&1; echo "prof32 rc=$?"
