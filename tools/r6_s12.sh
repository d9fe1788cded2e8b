#!/bin/bash
# round-6 session 12: the wgrad planner's automatic slot share (65 % at batch <= 32, 75 % at <= 64, 100 % above):
# the GPU suite, then same-box A/Bs against the old fixed 100 % at B=32, B=64, B=128 and the tube step
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
timeout -k 10 400 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/tests.log | tail -8
[ $rc -le 1 ] || exit $rc
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
step ab_b32 bash tools/ab3.sh 3 "auto:" "p100:AVT_WGRAD_SLOTS_PCT=100" "auto_def:AVT_WGRAD_DEFER=1"
cat gpurun_out/ab_b32.log
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 64"
step ab_b64 bash tools/ab3.sh 2 "auto:" "p100:AVT_WGRAD_SLOTS_PCT=100"
cat gpurun_out/ab_b64.log
export BENCH_ARGS="--traffic off --no-peaks --steps 20 --warmup 5"
step ab_b128 bash tools/ab3.sh 2 "auto:" "p85:AVT_WGRAD_SLOTS_PCT=85"
cat gpurun_out/ab_b128.log
export BENCH_ARGS="--traffic off --no-peaks --steps 10 --warmup 3 --workload tube"
step ab_tube bash tools/ab3.sh 2 "auto:" "p100:AVT_WGRAD_SLOTS_PCT=100"
cat gpurun_out/ab_tube.log
echo ALL_OK
