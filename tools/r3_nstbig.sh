#!/bin/bash
# Round 3: ring depth of the layer4 8-wave 256x256 wgrad tile (AVT_WGRAD_NST_BIG 3 default, 4)
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
BENCH_ARGS="--batch 32 --steps 30 --prof-steps 1" bash tools/ab3.sh 2 "nstbig3:" "nstbig4:AVT_WGRAD_NST_BIG=4" || exit 1
BENCH_ARGS="--steps 20 --prof-steps 1" bash tools/ab3.sh 2 "nstbig3:" "nstbig4:AVT_WGRAD_NST_BIG=4" || exit 1
