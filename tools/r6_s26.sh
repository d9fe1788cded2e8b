#!/bin/bash
# round-6 session 26: the BN backward reductions' block count (AVT_BN_RED_BLOCKS, default 512) at B=128 and B=32, with
# the BN tests first
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step t_bn env AVT_BN_RED_BLOCKS=1024 timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "bn" tests/test_model_gpu.py
tail -2 gpurun_out/t_bn.log
export BENCH_ARGS="--traffic off --no-peaks --steps 20 --warmup 5"
step ab_b128 bash tools/ab3.sh 2 "r512:" "r1024:AVT_BN_RED_BLOCKS=1024" "r768:AVT_BN_RED_BLOCKS=768"
cat gpurun_out/ab_b128.log
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
step ab_b32 bash tools/ab3.sh 2 "r512:" "r1024:AVT_BN_RED_BLOCKS=1024" "r256:AVT_BN_RED_BLOCKS=256"
cat gpurun_out/ab_b32.log
echo ALL_OK
