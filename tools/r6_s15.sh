#!/bin/bash
# round-6 session 15: the small-tile rule as a share of the CUs (AVT_SMALL_TILES_PCT, default 50: 64-row tiles only
# when the 128-row grid covers < 50 % of the CUs) vs never (0) and the old 100 %: the GPU suite, B=32, B=64, tube
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
timeout -k 10 400 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/tests.log | tail -8
[ $rc -le 1 ] || exit $rc
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
step ab_b32 bash tools/ab3.sh 3 "p50:" "p0:AVT_SMALL_TILES_PCT=0" "p100:AVT_SMALL_TILES_PCT=100" "p25:AVT_SMALL_TILES_PCT=25"
cat gpurun_out/ab_b32.log
export BENCH_ARGS="--traffic off --no-peaks --steps 10 --warmup 3 --workload tube"
step ab_tube bash tools/ab3.sh 2 "p50:" "p100:AVT_SMALL_TILES_PCT=100" "p0:AVT_SMALL_TILES_PCT=0"
cat gpurun_out/ab_tube.log
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 64"
step ab_b64 bash tools/ab3.sh 2 "p50:" "p0:AVT_SMALL_TILES_PCT=0"
cat gpurun_out/ab_b64.log
echo ALL_OK
