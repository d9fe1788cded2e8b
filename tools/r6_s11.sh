#!/bin/bash
# round-6 session 11: the wgrad planner's slot share (AVT_WGRAD_SLOTS_PCT) at B=64 (the N=4 shard of configs[2]) and a
# finer sweep at B=32, to place the size rule between B=32 (p50 +2 %) and B=128 (p50 -2 %)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 64"
step ab_b64 bash tools/ab3.sh 3 "p100:AVT_WGRAD_SLOTS_PCT=100" "p50:AVT_WGRAD_SLOTS_PCT=50" "p75:AVT_WGRAD_SLOTS_PCT=75"
cat gpurun_out/ab_b64.log
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
step ab_b32 bash tools/ab3.sh 2 "p100:AVT_WGRAD_SLOTS_PCT=100" "p50:AVT_WGRAD_SLOTS_PCT=50" "p35:AVT_WGRAD_SLOTS_PCT=35" "p65:AVT_WGRAD_SLOTS_PCT=65" "d50:AVT_WGRAD_SLOTS_PCT=50 AVT_WGRAD_DEFER=1"
cat gpurun_out/ab_b32.log
echo ALL_OK
