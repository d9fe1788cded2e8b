#!/bin/bash
# Round 3: wgrad split-K partials through slabs vs fp32 atomics, wave cost; B=32 and B=128.
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 2 "base:" "atom:AVT_WGRAD_SLAB_MAX=0" "wc8:AVT_WGRAD_WAVE_COST=8" "wc32:AVT_WGRAD_WAVE_COST=32" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 2 "base:" "atom:AVT_WGRAD_SLAB_MAX=0" || exit 1
# PMC stall breakdown of the layer3/4 halo kernels (B=128 shapes, fwd + dgrad): verdict r2 item 4
R=$(pwd); mkdir -p gpurun_out/pmc
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
C2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVES"
C3="GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for C in "$C1" "$C2" "$C3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/halo_p$i" -o run -- python "$R/tools/conv_bench.py" --only "l4 3x3" --kinds fwd,dgrad --variants 1 > gpurun_out/pmc/halo_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 gpurun_out/pmc/halo_p$i.log; exit 1; }
  echo "pmc pass $i ok"
done
