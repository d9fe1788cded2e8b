#!/bin/bash
# round-6 session 22: Conv3d weight pack through LDS rows: the pack and tube tests, kernel stats of the tube step, tube A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step t_tube timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_tube_gpu.py
tail -2 gpurun_out/t_tube.log
bash tools/gpu_check.sh "prof:r6tubep:--workload tube" > gpurun_out/prof.log 2>&1 || { tail -5 gpurun_out/prof.log; exit 1; }
grep -E "pack_conv3d" gpurun_out/kstats_r6tubep.txt | cut -c1-140
echo ALL_OK
