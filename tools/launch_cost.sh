#!/bin/bash
# Step cost of the forward BN finalize launches (AVT_DIAG_SKIP, graph only; timing only, wrong results):
# 1 = forward finalize, 2 = backward finalize, 4 = slab reduce left out (see the data-dependence caveat in
# avt_common.h: leaving out the forward finalize zeroes the activations)
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
BENCH_ARGS="--batch 32 --steps 30 --prof-steps 1" bash tools/ab3.sh 2 "all:" "-fin:AVT_DIAG_SKIP=1" "-bfin:AVT_DIAG_SKIP=2" "-slab:AVT_DIAG_SKIP=4" || exit 1
