#!/bin/bash
# Round 3: c64 forward BN partials: full-tile epilogue without per-element row tests: tests, stats-epilogue cost
# (tools/fin_probe.py forms B vs D), step A/B vs HEAD (libavt_base.so)
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
B=$(pwd)/audio-visual-tubes_amd/libavt_base.so
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "c64 or conv_fwd or model or hardway or fullsize or cfg" > gpurun_out/t_c64w.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/t_c64w.log; [ $rc -ne 0 ] && exit $rc
for lib in "$B" ""; do
for a in "--batch 128 --shape l1" "--batch 128 --shape al1" "--batch 128 --shape l3" "--batch 32 --shape l3"; do
env ${lib:+AVT_LIB_PATH=$lib} timeout -k 10 200 python tools/fin_probe.py $a > gpurun_out/fp.log 2>&1 || { tail -5 gpurun_out/fp.log; exit 1; }
echo "lib=${lib##*/}: $(grep 'us per link' gpurun_out/fp.log)"
done
done
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 2 "base:AVT_LIB_PATH=$B" "new:" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 2 "base:AVT_LIB_PATH=$B" "new:" || exit 1
