#!/bin/bash
# round-6 session 21: vectorised weight packs (16-byte dgrad transpose, wider fwd grid): parity tests, kernel stats, B=32 A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step t_pack timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pack" tests/test_schedule_gpu.py tests/test_model_gpu.py
tail -2 gpurun_out/t_pack.log
bash tools/gpu_check.sh "prof:r6b32p:--batch 32" > gpurun_out/prof.log 2>&1 || { tail -5 gpurun_out/prof.log; exit 1; }
grep -E "pack_(fwd|dgrad)_batched" gpurun_out/kstats_r6b32p.txt | cut -c1-140
echo ALL_OK
