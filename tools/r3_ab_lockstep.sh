#!/bin/bash
# Round 3: does the graph replay overlap the two trunks?  A/B of concurrency modes at B=32 / B=128 and a
# B=32 kernel trace with lockstep edges.
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$(pwd)
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 2 "c0:AVT_CONCURRENT=0" "c1:AVT_LOCKSTEP=0" "ls1:AVT_LOCKSTEP=1" "ls3:AVT_LOCKSTEP=3" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 1 "c0:AVT_CONCURRENT=0" "c1:AVT_LOCKSTEP=0" "ls1:AVT_LOCKSTEP=1" "ls3:AVT_LOCKSTEP=3" || exit 1
rm -rf gpurun_out/prof32
AVT_LOCKSTEP=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof32" -o run -- python "$R/bench.py" --batch 32 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof32.log 2>&1; echo "prof32 rc=$?"
