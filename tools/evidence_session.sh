#!/bin/bash
# The round's evidence in one GPU-box session (each GPU step under its own time limit; the first failure ends
# the session): determinism checks, the GPU suite + smoke, the benches (B=128 / B=32 with live PMC traffic and
# measured peaks, tube, two-view), kernel-stat profiles (concurrent and AVT_CONCURRENT=0), PMC passes over the
# layer3/4 halo convs.  usage: bash tools/evidence_session.sh  (outputs under gpurun_out/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 env REP_FRESH=w python -u tools/diag.py rep 32 14 14 512 512 60 > gpurun_out/rep1.log 2>&1 &&
timeout -k 10 300 env REP_FRESH=w python -u tools/diag.py rep 32 17 19 256 256 60 > gpurun_out/rep2.log 2>&1 &&
timeout -k 10 500 env DET_B=32 DET_FULL=1 DET_RUNS=3 python -u tools/diag.py runs > gpurun_out/det2_b32.log 2>&1 &&
bash tools/gpu_check.sh tests "bench:b128:--traffic-out gpurun_out/traffic_b128.json" \
  "bench:b32:--batch 32 --traffic-out gpurun_out/traffic_b32.json" "bench:tube:--workload tube" \
  "bench:twoview:--workload twoview" "prof:r5b128:" "prof:r5b32:--batch 32" &&
AVT_CONCURRENT=0 bash tools/gpu_check.sh "prof:r5b128serial:" &&
CB_ARGS="--only V.l3,V.l4,A.l4 --kinds fwd,dgrad --variants 1" bash tools/pmc.sh \
  "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
  "FETCH_SIZE" "WRITE_SIZE" "SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
