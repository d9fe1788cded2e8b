#!/bin/bash
# round-6 session 20: the 8-wave 256 x 128 halo tile for grids past one round of CUs (AVT_HALO8_PCT; the audio layer3
# GEMM's 324 tiles = 1.27 rounds lost 13 % alone on the chip in round 4) -- in the step, with the other trunk beside it
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
export BENCH_ARGS="--traffic off --no-peaks --steps 20 --warmup 5"
step ab_b128 bash tools/ab3.sh 3 "p100:" "p140:AVT_HALO8_PCT=140" "p200:AVT_HALO8_PCT=200"
cat gpurun_out/ab_b128.log
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 64"
step ab_b64 bash tools/ab3.sh 2 "p100:" "p140:AVT_HALO8_PCT=140" "p200:AVT_HALO8_PCT=200"
cat gpurun_out/ab_b64.log
echo ALL_OK
