#!/bin/bash
# round-6 session 25: layer-1 c64 dgrad epilogue with the tile's residual / mask loads hoisted (one round trip per tile):
# c64 + model tests, serial kernel stats at B=128 and B=32 (compare conv_c64_kernel<1, 2, 8>)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step t_c64 timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "c64 or conv_dgrad or bn_bwd_mask" tests/test_model_gpu.py tests/test_fullsize_gpu.py
tail -2 gpurun_out/t_c64.log
AVT_CONCURRENT=0 bash tools/gpu_check.sh "prof:r6b128c:" "prof:r6b32c:--batch 32" > gpurun_out/prof.log 2>&1 || { tail -5 gpurun_out/prof.log; exit 1; }
grep -E "c64_kernel" gpurun_out/kstats_r6b128c.txt gpurun_out/kstats_r6b32c.txt | cut -c1-150
echo ALL_OK
