#!/bin/bash
# Round 3: wgrad split policy sweep at the B=32 shard size (slab on), per shape
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python tools/conv_bench.py --batch 32 --kinds wgrad --variants 1 --wgrad-policy "0,4;96,4;128,4;192,4;256,4;384,4;512,4" --wgrad-tiles 1,0 2>&1 | grep -v "amdgpu" || exit 1
