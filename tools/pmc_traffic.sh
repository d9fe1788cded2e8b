#!/bin/bash
# HBM traffic of the conv family (and every other kernel) of the bench workload, from PMC
# counters: one rocprofv3 pass for FETCH_SIZE, one for WRITE_SIZE (they do not fit one pass on
# gfx950), kernel-trace only.  Eager launches (--no-graph), 1 warm-up + 1 timed step.
# usage: bash tools/pmc_traffic.sh [extra bench.py args]; summary: python tools/traffic_summary.py
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf "gpurun_out/traffic/$ctr"
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$R/gpurun_out/traffic/$ctr" -o run -- \
    python "$R/bench.py" --steps 1 --warmup 1 --no-graph --prof-steps 0 --no-cpu-baseline "$@" \
    > "gpurun_out/traffic/$ctr.log" 2>&1 || { echo "pass $ctr failed"; tail -5 "gpurun_out/traffic/$ctr.log"; exit 1; }
  echo "pass $ctr ok"
done
python tools/traffic_summary.py gpurun_out/traffic 2 --json gpurun_out/traffic/conv_traffic.json > gpurun_out/traffic/summary.txt && cat gpurun_out/traffic/summary.txt
