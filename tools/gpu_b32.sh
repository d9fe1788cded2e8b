#!/bin/bash
# full GPU tests, then the B=32 (configs[2] per-GPU shard) bench + rocprof kernel stats
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --batch 32 --steps 20 --no-cpu-baseline > gpurun_out/bench_b32.log 2>&1; rc=$?; tail -1 gpurun_out/bench_b32.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof32
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof32" -o run -- python "$R/bench.py" --batch 32 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof32.log 2>&1; echo "prof rc=$?"
