#!/bin/bash
# What bounds the halo fwd/dgrad: the -DAVT_DIAG build (tools/build_variant.sh libavt_diag.so -DAVT_DIAG) run
# with AVT_HALO_DBG bits (conv_halo.h: 1 weight DMA out of range, 2 patch DMA out of range, 4 no per-tap barrier,
# 8 no MFMA, 16 no epilogue stores) over the layer2-4 3x3 shapes.  usage: bash tools/halo_diag.sh [bits...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for d in "${@:-0 1 2 3 4 8 16}"; do
  AVT_LIB_PATH=$R/audio-visual-tubes_amd/libavt_diag.so AVT_HALO_DBG=$d timeout -k 10 300 python tools/conv_bench.py \
    --kinds fwd,dgrad --variants 1 --only "l2 3x3,l3 3x3,l4 3x3" $CB_ARGS > gpurun_out/halo_diag_$d.log 2>&1 || \
    { echo "diag $d failed"; tail -3 gpurun_out/halo_diag_$d.log; exit 1; }
  echo "== AVT_HALO_DBG=$d"; grep -v amdgpu.ids gpurun_out/halo_diag_$d.log | tail -16
done
