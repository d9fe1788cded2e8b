# One box session: determinism checks after a kernel change, the full GPU suite + smoke, then the evidence runs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 env REP_FRESH=w python -u tools/diag_rep.py 32 14 14 512 512 60 > gpurun_out/rep1.log 2>&1 &&
timeout -k 10 300 env REP_FRESH=w python -u tools/diag_rep.py 32 17 19 256 256 60 > gpurun_out/rep2.log 2>&1 &&
timeout -k 10 500 env DET_B=32 DET_FULL=1 DET_RUNS=3 python -u tools/diag_det2.py > gpurun_out/det2_b32.log 2>&1 &&
bash tools/gpu_check.sh tests "bench:b128:--traffic-out gpurun_out/traffic_b128.json" \
  "bench:b32:--batch 32 --traffic-out gpurun_out/traffic_b32.json" "prof:r4b128:" "prof:r4b32:--batch 32" &&
AVT_CONCURRENT=0 bash tools/gpu_check.sh "prof:r4b128serial:"
