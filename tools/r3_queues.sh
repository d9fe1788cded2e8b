#!/bin/bash
# Round 3: does a third graph branch (overlapped Adam / wgrad streams) serialize the two trunk branches on
# the 4 default HW queues?  Step A/B at B=32 with GPU_MAX_HW_QUEUES 4 / 8; wgrad split policy sweep.
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 2 "old:" "oldq8:GPU_MAX_HW_QUEUES=8" "adam:AVT_ADAM_OVERLAP=1" "adamq8:AVT_ADAM_OVERLAP=1 GPU_MAX_HW_QUEUES=8" "ws2q8:AVT_ADAM_OVERLAP=1 AVT_WGRAD_STREAMS=2 GPU_MAX_HW_QUEUES=8" "ws1q8:AVT_ADAM_OVERLAP=1 AVT_WGRAD_STREAMS=1 GPU_MAX_HW_QUEUES=8" "ws2q16:AVT_ADAM_OVERLAP=1 AVT_WGRAD_STREAMS=2 GPU_MAX_HW_QUEUES=16" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 1 "old:" "oldq8:GPU_MAX_HW_QUEUES=8" "adamq8:AVT_ADAM_OVERLAP=1 GPU_MAX_HW_QUEUES=8" "ws2q8:AVT_ADAM_OVERLAP=1 AVT_WGRAD_STREAMS=2 GPU_MAX_HW_QUEUES=8" || exit 1
for B in 32 128; do
for sm in "32,16" "256,16"; do
timeout -k 10 400 python tools/conv_bench.py --batch $B --kinds wgrad --variants 1 --slab-max $sm --wgrad-policy "0,4;128,4;256,4;384,4;512,4;768,4;1024,4" > gpurun_out/cbw.txt 2>&1 || { tail -5 gpurun_out/cbw.txt; exit 1; }
echo "== B=$B slab-max $sm"; grep -v amdgpu gpurun_out/cbw.txt
done; done
