#!/bin/bash
# Round 3: same-box A/B of HEAD against the mid-round profile commit 1843188 (libavt_base.so)
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
B=$(pwd)/audio-visual-tubes_amd/libavt_base.so
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 3 "1843188:AVT_LIB_PATH=$B" "HEAD:" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 3 "1843188:AVT_LIB_PATH=$B" "HEAD:" || exit 1
