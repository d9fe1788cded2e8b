#!/bin/bash
# round-6 session 27: each trunk's layer4+3 Adam update on a side stream beside its layer2..stem backward
# (AVT_ADAM_HI=1): the step / schedule tests under it, then same-box A/Bs at B=32 and B=128
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step t_adam env AVT_ADAM_HI=1 timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_model_gpu.py tests/test_schedule_gpu.py tests/test_fullsize_gpu.py
tail -2 gpurun_out/t_adam.log
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
step ab_b32 bash tools/ab3.sh 3 "base:" "adamhi:AVT_ADAM_HI=1"
cat gpurun_out/ab_b32.log
export BENCH_ARGS="--traffic off --no-peaks --steps 20 --warmup 5"
step ab_b128 bash tools/ab3.sh 3 "base:" "adamhi:AVT_ADAM_HI=1"
cat gpurun_out/ab_b128.log
echo ALL_OK
