#!/bin/bash
# round-6 session 2: Conv3d halo form (tube tests, per-shape bench, tube-step A/B), halo barrier / DMA ablation
# (-DAVT_DIAG halo_bench: dbg 4 = no per-step barrier, 3 = no DMA traffic; wrong results, timing only)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
soft() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; [ $rc -eq 0 ] || tail -25 "gpurun_out/$name.log"; }
step dconv3d timeout -k 10 200 python tools/diag_conv3d.py
soft hdiag4 timeout -k 10 120 tools/halo_bench_diag 128 2 20 x 4
soft hdiag3 timeout -k 10 120 tools/halo_bench_diag 128 2 20 x 3
export BENCH_ARGS="--workload tube --traffic off --no-peaks --steps 10 --warmup 3"
step ab_tube bash tools/ab3.sh 2 "halo3d:AVT_HALO3D=1" "gather:AVT_HALO3D=0"
echo ALL_OK
