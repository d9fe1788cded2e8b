#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python tools/conv_bench.py --variants 1 --kinds fwd,dgrad --only "l2" --halo 1,2 2>&1 | grep -v amdgpu
timeout -k 10 200 python tools/conv_bench.py --variants 1 --kinds fwd,dgrad --only "l2" --halo 1,2 --batch 32 2>&1 | grep -v amdgpu
timeout -k 10 200 python tools/conv_bench.py --variants 1 --kinds fwd,dgrad --only "l3" --halo 1,2 --batch 32 --small 1,0 2>&1 | grep -v amdgpu
timeout -k 10 200 python tools/conv_bench.py --variants 1 --kinds fwd,dgrad --only "l4" --halo 1,2 --batch 32 --small 1,0 2>&1 | grep -v amdgpu
