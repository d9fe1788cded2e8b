#!/bin/bash
# the round-6 evidence session (tools/r6_final.sh), then -- soft, after the evidence -- the deferred batched wgrad
# reduce's parity tests and a B=32 A/B (AVT_WGRAD_DEFER, off by default until measured)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/r6_final.sh || exit $?
timeout -k 10 400 env AVT_WGRAD_DEFER=1 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  "tests/test_kernels_gpu.py::test_wgrad_deferred_batched_reduce" tests/test_model_gpu.py tests/test_ddp_gpu.py \
  > gpurun_out/t_defer.log 2>&1; rc=$?
echo "t_defer rc=$rc"; tail -3 gpurun_out/t_defer.log
[ $rc -le 1 ] || exit $rc
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
bash tools/ab3.sh 2 "defer:AVT_WGRAD_DEFER=1" "each:AVT_WGRAD_DEFER=0" > gpurun_out/ab_defer_b32.log 2>&1
cat gpurun_out/ab_defer_b32.log
echo ALL_DONE
