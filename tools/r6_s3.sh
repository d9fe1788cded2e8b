#!/bin/bash
# round-6 session 3: Conv3d halo + two-tap halo in libavt: parity tests, the Conv3d tap-gather triangulation,
# per-shape benches, step A/Bs (B=128: AVT_HALO_TPS2 1 vs 0; tube: AVT_HALO3D 1 vs 0)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
soft() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; [ $rc -eq 0 ] || tail -25 "gpurun_out/$name.log"; }
soft t_tube timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_tube_gpu.py \
  "tests/test_kernels_gpu.py::test_halo8_form_and_ring_bitwise_equal"
step dconv3d timeout -k 10 200 python tools/diag_conv3d.py
step c3d timeout -k 10 200 env AVT_HALO_TPS2=1 python tools/conv3d_bench.py --halo3d 1,0
step c3d0 timeout -k 10 200 env AVT_HALO_TPS2=0 python tools/conv3d_bench.py --halo3d 1,2
export BENCH_ARGS="--traffic off --no-peaks --steps 20 --warmup 5"
step ab_b128 bash tools/ab3.sh 3 "tps2:AVT_HALO_TPS2=1" "one:AVT_HALO_TPS2=0"
export BENCH_ARGS="--workload tube --traffic off --no-peaks --steps 10 --warmup 3"
step ab_tube bash tools/ab3.sh 2 "halo3d:AVT_HALO3D=1" "gather:AVT_HALO3D=0"
soft hdiag4 timeout -k 10 120 tools/halo_bench_diag 128 2 20 x 4
soft hdiag3 timeout -k 10 120 tools/halo_bench_diag 128 2 20 x 3
echo ALL_OK
