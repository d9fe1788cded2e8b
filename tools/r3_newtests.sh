#!/bin/bash
# Round 3: the new boundary tests (DataParallel replica, deepcopy, standalone HardWayAttention), then the
# concurrency A/B (tools/r3_ab_lockstep.sh).
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_boundary_gpu.py tests/test_tube_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k "dataparallel or attention or deepcopy" > gpurun_out/t_new.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t_new.log | tail -12; [ $rc -ne 0 ] && exit $rc
bash tools/r3_ab_lockstep.sh
