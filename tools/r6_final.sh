#!/bin/bash
# Round-6 evidence in one GPU-box session (each GPU step under its own time limit; the first failure ends the session):
# the GPU suite + smoke, the benches (B=128 and B=32 with live PMC traffic and measured peaks, tube, two-view), kernel
# stats (B=128 concurrent and serial, B=32, tube), determinism at B=32.  Outputs under gpurun_out/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
MAXFAIL=5 bash tools/gpu_check.sh tests "bench:b128:--traffic-out gpurun_out/traffic_b128.json" \
  "bench:b32:--batch 32 --traffic-out gpurun_out/traffic_b32.json" "bench:tube:--workload tube" \
  "bench:twoview:--workload twoview" "prof:r6b128:" "prof:r6b32:--batch 32" "prof:r6tube:--workload tube" &&
AVT_CONCURRENT=0 bash tools/gpu_check.sh "prof:r6b128serial:" &&
timeout -k 10 500 env DET_B=32 DET_FULL=1 DET_RUNS=3 python -u tools/diag.py runs > gpurun_out/det_b32.log 2>&1 &&
echo EVIDENCE_OK
