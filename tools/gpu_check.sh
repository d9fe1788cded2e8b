#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel stats.  Each GPU step has its own
# time limit; a crash/timeout (rc > 1) stops the script before any further GPU work.
# usage: bash tools/gpu_check.sh [tests|bench|prof|all]
what=${1:-all}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
rc=0
if [ "$what" = all ] || [ "$what" = tests ]; then
  timeout -k 10 900 python -u -m pytest ${AVT_TESTS:-tests} -x -v -s -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -8
  [ $rc -gt 1 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ "$what" = all ] || [ "$what" = bench ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ "$what" = all ] || [ "$what" = prof ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
    python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?
  echo "prof rc=$rc"; tail -1 gpurun_out/prof.log
fi
exit $rc
