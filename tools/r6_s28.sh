#!/bin/bash
# round-6 session 28: HIP hardware queues per process (GPU_MAX_HW_QUEUES, 4 on the box) for the two-stream captured step
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
step ab_b32 bash tools/ab3.sh 2 "q4:GPU_MAX_HW_QUEUES=4" "q8:GPU_MAX_HW_QUEUES=8" "q2:GPU_MAX_HW_QUEUES=2"
cat gpurun_out/ab_b32.log
export BENCH_ARGS="--traffic off --no-peaks --steps 20 --warmup 5"
step ab_b128 bash tools/ab3.sh 2 "q4:GPU_MAX_HW_QUEUES=4" "q8:GPU_MAX_HW_QUEUES=8"
cat gpurun_out/ab_b128.log
echo ALL_OK
