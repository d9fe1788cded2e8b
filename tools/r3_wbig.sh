#!/bin/bash
# Round 3: layer4 wgrad 8-wave 256x256 tile (AVT_WGRAD_BIG=1) vs 4-wave tiles, B=32 and B=128
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 2 "big1:" "big0:AVT_WGRAD_BIG=0" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 2 "big1:" "big0:AVT_WGRAD_BIG=0" || exit 1
