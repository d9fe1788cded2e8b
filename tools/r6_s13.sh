#!/bin/bash
# round-6 session 13: with the wgrad planner's shared-chip slot share in place, the fwd/dgrad small-tile rule
# (AVT_SMALL_TILES: 64-row tiles when the 128-row grid has fewer than N blocks per CU; default 1) at B=32 and B=64
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
step ab_b32 bash tools/ab3.sh 3 "st1:" "st0:AVT_SMALL_TILES=0" "st2:AVT_SMALL_TILES=2"
cat gpurun_out/ab_b32.log
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 64"
step ab_b64 bash tools/ab3.sh 2 "st1:" "st0:AVT_SMALL_TILES=0"
cat gpurun_out/ab_b64.log
echo ALL_OK
