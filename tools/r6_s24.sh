#!/bin/bash
# round-6 session 24: the head GEMM with double-buffered LDS tiles (one barrier per k-tile): head / model / two-view /
# tube tests, kernel stats at B=128 and B=32
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step t_head timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "hardway or head or sgemm" tests/test_model_gpu.py tests/test_twoview_gpu.py
tail -2 gpurun_out/t_head.log
bash tools/gpu_check.sh "prof:r6b128h:" "prof:r6b32h:--batch 32" > gpurun_out/prof.log 2>&1 || { tail -5 gpurun_out/prof.log; exit 1; }
grep -E "sgemm" gpurun_out/kstats_r6b128h.txt gpurun_out/kstats_r6b32h.txt | cut -c1-170
echo ALL_OK
