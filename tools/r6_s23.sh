#!/bin/bash
# round-6 session 23: remaining tile knobs at B=32 under the shared-chip defaults
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
step ab_b32 bash tools/ab3.sh 2 "base:" "big0:AVT_WGRAD_BIG=0" "kg1:AVT_WGRAD_KG=1" "snst4:AVT_HALO_SMALL_NST=4" "h8nst4:AVT_HALO8_NST=4" "nst6:AVT_WGRAD_NST=6"
cat gpurun_out/ab_b32.log
echo ALL_OK
