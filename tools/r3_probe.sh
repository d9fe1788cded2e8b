#!/bin/bash
# Round 3: host enqueue time of a graph replay vs its GPU time, B=32 and B=128
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python tools/launch_probe.py --batch 32 --reps 10 > gpurun_out/probe.log 2>&1 || { tail -5 gpurun_out/probe.log; exit 1; }
timeout -k 10 240 python tools/launch_probe.py --batch 128 --reps 10 >> gpurun_out/probe.log 2>&1 || { tail -5 gpurun_out/probe.log; exit 1; }
grep "B=" gpurun_out/probe.log
