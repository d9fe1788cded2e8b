#!/bin/bash
# round-6 session 9: the wgrad split planner assuming a share of the chip (AVT_WGRAD_SLOTS_PCT; the other trunk's
# kernels run beside it): fewer splits -> fewer slab partials and shorter reduces.  Same-box A/Bs at B=32 and B=128
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
step ab_b32 bash tools/ab3.sh 3 "p100:AVT_WGRAD_SLOTS_PCT=100" "p50:AVT_WGRAD_SLOTS_PCT=50" "p25:AVT_WGRAD_SLOTS_PCT=25"
cat gpurun_out/ab_b32.log
export BENCH_ARGS="--traffic off --no-peaks --steps 20 --warmup 5"
step ab_b128 bash tools/ab3.sh 2 "p100:AVT_WGRAD_SLOTS_PCT=100" "p50:AVT_WGRAD_SLOTS_PCT=50"
cat gpurun_out/ab_b128.log
echo ALL_OK
