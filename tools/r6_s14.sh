#!/bin/bash
# round-6 session 14: small tiles off (AVT_SMALL_TILES=0: +1.6 % at B=32, +0.5 % at B=64 in session 13) with the
# 128-row halo split-K's block target (AVT_SPLITK_BLOCKS, default 2 per CU) or split-K off; the tube and B=128 checks
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
step ab_b32 bash tools/ab3.sh 2 "st0:AVT_SMALL_TILES=0" "st0_b256:AVT_SMALL_TILES=0 AVT_SPLITK_BLOCKS=256" "st0_nosplit:AVT_SMALL_TILES=0 AVT_HALO_SPLITK=1" "st0_b384:AVT_SMALL_TILES=0 AVT_SPLITK_BLOCKS=384"
cat gpurun_out/ab_b32.log
step ab_b32s bash tools/ab3.sh 3 "st0:AVT_SMALL_TILES=0" "c64_75:AVT_SMALL_TILES=0 AVT_C64_SHARE=75" "hw65:AVT_SMALL_TILES=0 AVT_WGRAD_HALO_SHARE=65" "c50:AVT_SMALL_TILES=0 AVT_C64_SHARE=50"
cat gpurun_out/ab_b32s.log
export BENCH_ARGS="--traffic off --no-peaks --steps 10 --warmup 3 --workload tube"
step ab_tube bash tools/ab3.sh 2 "st1:" "st0:AVT_SMALL_TILES=0"
cat gpurun_out/ab_tube.log
export BENCH_ARGS="--traffic off --no-peaks --steps 20 --warmup 5"
step ab_b128 bash tools/ab3.sh 2 "st1:" "st0:AVT_SMALL_TILES=0"
cat gpurun_out/ab_b128.log
echo ALL_OK
