# Round-4 evidence, second session: tube and two-view benches, PMC passes over the layer3/4 halo fwd/dgrad.
set -o pipefail
bash tools/gpu_check.sh "bench:tube:--workload tube" "bench:twoview:--workload twoview" &&
CB_ARGS="--only V.l3,V.l4,A.l4 --kinds fwd,dgrad --variants 1" bash tools/pmc.sh \
  "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
  "FETCH_SIZE" "WRITE_SIZE" "SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
