#!/bin/bash
# round-6 session 10: the wgrad slab reduces deferred to one batched launch per trunk segment (AVT_WGRAD_DEFER) and the
# planner's slot share (AVT_WGRAD_SLOTS_PCT): parity tests, then same-box A/Bs at B=32 and B=128
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step t_defer timeout -k 10 500 env AVT_WGRAD_DEFER=1 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_kernels_gpu.py::test_wgrad_deferred_batched_reduce" tests/test_model_gpu.py \
  tests/test_ddp_gpu.py tests/test_fullsize_gpu.py tests/test_twoview_gpu.py tests/test_boundary_gpu.py
tail -2 gpurun_out/t_defer.log
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
step ab_b32 bash tools/ab3.sh 3 "defer:AVT_WGRAD_DEFER=1" "each:AVT_WGRAD_DEFER=0" "defer_p50:AVT_WGRAD_DEFER=1 AVT_WGRAD_SLOTS_PCT=50"
cat gpurun_out/ab_b32.log
export BENCH_ARGS="--traffic off --no-peaks --steps 20 --warmup 5"
step ab_b128 bash tools/ab3.sh 2 "defer:AVT_WGRAD_DEFER=1" "each:AVT_WGRAD_DEFER=0"
cat gpurun_out/ab_b128.log
echo ALL_OK
