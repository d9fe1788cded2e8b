#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
for d in 0 1 2 3; do
  AVT_C64_DBG=$d timeout -k 10 120 python tools/conv_bench.py --only l1 --variants 1 --kinds fwd,dgrad 2>&1 | grep -v amdgpu | sed "s/^/dbg=$d /" | head -2 || exit 1
done
AVT_C64=0 timeout -k 10 120 python tools/conv_bench.py --only l1 --variants 1 --kinds fwd,dgrad 2>&1 | grep -v amdgpu | sed "s/^/c64off /" | head -2
