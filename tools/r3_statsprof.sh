#!/bin/bash
# Round 3: rocprof kernel stats of the B=128 graph step with real vs dummy forward-finalize outputs
# (AVT_DIAG_SKIP=16, timing only) -- which kernels pay for the finalize's stats writes
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$(pwd)
for v in 0 16; do
rm -rf gpurun_out/sp$v
AVT_DIAG_SKIP=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/sp$v" -o run -- python "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --prof-steps 1 > gpurun_out/sp$v.log 2>&1; rc=$?; echo "prof $v rc=$rc"; tail -1 gpurun_out/sp$v.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
done
exit 0
