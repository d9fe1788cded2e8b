#!/bin/bash
# round-6 session 4: Conv3d halo defaults (layer1-4) -- tube parity tests, the case7 triangulation, tube-step A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
soft() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; [ $rc -eq 0 ] || tail -25 "gpurun_out/$name.log"; }
soft t_tube timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_tube_gpu.py \
  "tests/test_kernels_gpu.py::test_halo8_form_and_ring_bitwise_equal" tests/test_fullsize_gpu.py
soft t_case7 timeout -k 10 200 python -u -m pytest -v --timeout 100 --timeout-method thread "tests/test_tube_gpu.py::test_conv3d_fwd_and_bn_stats[case7-0]"
step dconv3d timeout -k 10 200 python tools/diag_conv3d.py
export BENCH_ARGS="--workload tube --traffic off --no-peaks --steps 10 --warmup 3"
step ab_tube bash tools/ab3.sh 2 "halo3d2:AVT_HALO3D=2" "halo3d1:AVT_HALO3D=1" "gather:AVT_HALO3D=0"
echo ALL_OK
