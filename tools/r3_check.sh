#!/bin/bash
# Round 3 checkpoint: full GPU suite (full-size diagnostics printed), bench B=128 / B=32, B=32 kernel stats.
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -12; [ $rc -gt 1 ] && exit $rc
grep -E "NORM EXCEEDS|DIRECTION BELOW|gradient direction" gpurun_out/gpu_tests.log | head -40
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --batch 32 --steps 30 --no-cpu-baseline > gpurun_out/bench_b32.log 2>&1; rc=$?; echo "b32 rc=$rc"; tail -1 gpurun_out/bench_b32.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof32
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof32" -o run -- python "$R/bench.py" --batch 32 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof32.log 2>&1; echo "prof32 rc=$?"
python tools/timeline.py gpurun_out/prof32/run_kernel_trace.csv --top 40 > gpurun_out/timeline32.txt 2>&1; echo "timeline rc=$?"
