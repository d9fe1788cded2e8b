#!/bin/bash
# GPU pytest selection with its own time limit: bash tools/gpu_tests.sh <pytest args...>
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu "$@" \
  > gpurun_out/gpu_sel.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|error" gpurun_out/gpu_sel.log | tail -40
exit $rc
