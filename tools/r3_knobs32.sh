#!/bin/bash
# Round 3: B=32 sweep of planner knobs (small-tile threshold, wgrad wave cost, slab limit)
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
BENCH_ARGS="--batch 32 --steps 30 --prof-steps 1" bash tools/ab3.sh 2 "default:" "small2:AVT_SMALL_TILES=2" "wcost8:AVT_WGRAD_WAVE_COST=8" "wcost24:AVT_WGRAD_WAVE_COST=24" "slab16:AVT_WGRAD_SLAB_MAX=16" || exit 1
