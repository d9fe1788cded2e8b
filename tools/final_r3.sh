#!/bin/bash
# Round-3 evidence run: full GPU tests, smoke, bench (B=128), rocprof kernel stats, PMC HBM traffic
# (two passes), B=32 bench.  Each GPU step has its own limit; the first failure ends the script.
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash tools/pmc_traffic.sh > gpurun_out/traffic.log 2>&1; rc=$?; echo "traffic rc=$rc"; head -4 gpurun_out/traffic/summary.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --batch 32 --steps 20 --no-cpu-baseline > gpurun_out/bench_b32.log 2>&1; rc=$?; echo "b32 rc=$rc"; tail -1 gpurun_out/bench_b32.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof32
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof32" -o run -- python "$R/bench.py" --batch 32 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof32.log 2>&1; rc=$?; echo "prof32 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload tube --no-cpu-baseline > gpurun_out/bench_tube.log 2>&1; rc=$?; echo "tube rc=$rc"; tail -1 gpurun_out/bench_tube.log | cut -c1-120; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload twoview --no-cpu-baseline > gpurun_out/bench_twoview.log 2>&1; rc=$?; echo "twoview rc=$rc"; tail -1 gpurun_out/bench_twoview.log | cut -c1-120
exit $rc
