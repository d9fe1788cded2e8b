#!/bin/bash
# Round 3: new boundary tests + halo-stage bitwise test + full-size direction checks (informational),
# halo stage sweep (conv_bench B=32 / B=128), then the concurrency A/B.
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_boundary_gpu.py tests/test_tube_gpu.py tests/test_kernels_gpu.py tests/test_fullsize_gpu.py -v -s --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k "dataparallel or attention or deepcopy or halo_stages or fullsize or cfg4" > gpurun_out/t_new.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t_new.log | tail -16; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/conv_bench.py --batch 32 --only "l3 3x3" --kinds fwd --stages "2,2;2,3;2,4;2,5" --variants 1 2>&1 | grep -v "^{" || exit 1
timeout -k 10 300 python tools/conv_bench.py --batch 32 --only "l4" --kinds fwd --stages "2,2;2,3;2,4;2,5" --variants 1 2>&1 | grep -v "^{" || exit 1
timeout -k 10 300 python tools/conv_bench.py --batch 128 --only "l4" --kinds fwd --stages "2,2;3,2" --variants 1 2>&1 | grep -v "^{" || exit 1
timeout -k 10 300 python tools/conv_bench.py --batch 128 --only "l3 3x3" --kinds fwd --stages "2,2;3,2" --variants 1 2>&1 | grep -v "^{" || exit 1
bash tools/r3_ab_lockstep.sh
