#!/bin/bash
# round-6 session 8: the wgrad split-K slab summed inside the wgrad kernel (avt_conv2d_wgrad_tk, AVT_WGRAD_FUSED):
# parity tests, then same-box A/Bs at B=32 and B=128
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step t_fused timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -s \
  "tests/test_kernels_gpu.py::test_conv_wgrad_fused_reduce" "tests/test_kernels_gpu.py::test_conv_wgrad" \
  tests/test_model_gpu.py tests/test_ddp_gpu.py
grep "fused - separate" gpurun_out/t_fused.log | head -60
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
step ab_b32 bash tools/ab3.sh 3 "fused:AVT_WGRAD_FUSED=1" "sep:AVT_WGRAD_FUSED=0"
cat gpurun_out/ab_b32.log
export BENCH_ARGS="--traffic off --no-peaks --steps 20 --warmup 5"
step ab_b128 bash tools/ab3.sh 2 "fused:AVT_WGRAD_FUSED=1" "sep:AVT_WGRAD_FUSED=0"
cat gpurun_out/ab_b128.log
echo ALL_OK
