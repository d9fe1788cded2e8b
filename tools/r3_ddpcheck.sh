#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
for sp in 1 0 1; do
AVT_SPLIT_PACK=$sp timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "matches_dp_mean" > gpurun_out/t_ddp$sp.log 2>&1; echo "split_pack=$sp rc=$?"; grep -E "passed|failed|ACTUAL|DESIRED" gpurun_out/t_ddp$sp.log | tail -4
done
