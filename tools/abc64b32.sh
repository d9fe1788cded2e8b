#!/bin/bash
# layer-1 convs at small batch: c64 (8 / 4 waves) vs the tap-gather/halo kernels, per shape and in the B=32 step
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
for b in 32 64; do for v in "AVT_C64=1" "AVT_C64=1 AVT_C64_WAVES=4" "AVT_C64=0"; do env $v timeout -k 10 200 python tools/conv_bench.py --batch $b --only l1 --variants 1 --kinds fwd,dgrad 2>&1 | grep -E "l1 " | sed "s/^/b$b $v /" || exit 1; done; done
BENCH_ARGS="--batch 32 --steps 20" bash tools/ab3.sh 3 "c64:AVT_C64=1" "gather:AVT_C64=0"
