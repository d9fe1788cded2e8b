#!/bin/bash
# Step cost of the small launch classes (AVT_DIAG_SKIP: left out of the captured graph only; timing
# only, wrong results) and of the serial step prologue (AVT_VISION_PRE): B=32 and B=128
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
BENCH_ARGS="--batch 32 --steps 30 --prof-steps 1" bash tools/ab3.sh 2 "all:" "pre0:AVT_VISION_PRE=0" "-fin:AVT_DIAG_SKIP=1" "-bfin:AVT_DIAG_SKIP=2" "-slab:AVT_DIAG_SKIP=4" "-all3:AVT_DIAG_SKIP=7" || exit 1
BENCH_ARGS="--steps 20 --prof-steps 1" bash tools/ab3.sh 2 "all:" "pre0:AVT_VISION_PRE=0" "-fin:AVT_DIAG_SKIP=1" "-all3:AVT_DIAG_SKIP=7" || exit 1
