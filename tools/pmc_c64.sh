#!/bin/bash
# PMC stall breakdown of the layer-1 conv kernels (one shape, dgrad): c64 normal / no memory (dbg 3)
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
R=$(pwd)
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for d in 0 3; do
  AVT_C64_DBG=$d timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/c64_$d" -o run -- python "$R/tools/conv_bench.py" --only "V.l1" --kinds dgrad --variants 1 > gpurun_out/pmc/c64_$d.log 2>&1 || { echo "pass $d failed"; tail -5 gpurun_out/pmc/c64_$d.log; exit 1; }
  echo "pass $d ok"; grep -v amdgpu gpurun_out/pmc/c64_$d.log | grep TFLOP
done
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/c64_clk" -o run -- python "$R/tools/conv_bench.py" --only "V.l1" --kinds dgrad --variants 1 > gpurun_out/pmc/c64_clk.log 2>&1; echo "clk rc=$?"
