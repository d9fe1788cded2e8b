#!/bin/bash
# round-6 session 17: the R3D stem max-pool tests, then B=128 knob re-checks under the shared-chip defaults
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
step t_mp timeout -k 10 300 python -u -m pytest tests/test_tube_gpu.py -q -x --timeout 120 --timeout-method thread -k "maxpool or r3d_forward" -s
grep -E "rel err|passed|failed" gpurun_out/t_mp.log
export BENCH_ARGS="--traffic off --no-peaks --steps 20 --warmup 5"
step ab_b128 bash tools/ab3.sh 2 "base:" "tps2:AVT_HALO_TPS2=1" "sl90:AVT_WGRAD_SLOTS_PCT=90" "c64_90:AVT_C64_SHARE=90"
cat gpurun_out/ab_b128.log
echo ALL_OK
