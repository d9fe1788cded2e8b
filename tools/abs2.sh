#!/bin/bash
# stride-2 dgrad classes in one launch vs four: kernel tests, per-shape dgrad (B=128, B=32), step A/B at B=128 and B=32
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider -k "dgrad or strided" > gpurun_out/k.log 2>&1; rc=$?; tail -1 gpurun_out/k.log; [ $rc -ne 0 ] && { grep -E "^(FAILED|E )" gpurun_out/k.log | head -30; exit $rc; }
for b in 128 32; do for o in 0 1; do AVT_S2_ONE=$o timeout -k 10 200 python tools/conv_bench.py --batch $b --variants 1 --kinds dgrad 2>&1 | grep -E "s2 " | sed "s/^/b$b one$o /"; done; done
bash tools/ab3.sh 3 "four:AVT_S2_ONE=0" "one:AVT_S2_ONE=1" && BENCH_ARGS="--batch 32 --steps 20" bash tools/ab3.sh 3 "four32:AVT_S2_ONE=0" "one32:AVT_S2_ONE=1"
