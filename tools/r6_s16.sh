#!/bin/bash
# round-6 session 16: under the shared-chip planner rules, the wgrad split knobs at B=32: the layer-1 halo wgrad's
# minimum k-tiles per split (AVT_ROW3_MIN_KT, default 8) and the TN planner's per-block fixed cost (AVT_WGRAD_WAVE_COST, 16)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
step ab_b32 bash tools/ab3.sh 3 "base:" "r3kt16:AVT_ROW3_MIN_KT=16" "wc32:AVT_WGRAD_WAVE_COST=32" "wc8:AVT_WGRAD_WAVE_COST=8" "r3kt4:AVT_ROW3_MIN_KT=4"
cat gpurun_out/ab_b32.log
echo ALL_OK
