#!/bin/bash
# Round 3: where a BN finalize's step cost comes from (tools/fin_probe.py), one and two streams
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
for a in "--batch 128 --shape l1 --streams 2 --shape2 al1" "--batch 128 --shape l3 --streams 2 --shape2 al3" "--batch 32 --shape l1 --streams 2 --shape2 al1" "--batch 32 --shape l3 --streams 2 --shape2 al3"; do
timeout -k 10 200 python tools/fin_probe.py $a > gpurun_out/fp.log 2>&1 || { tail -5 gpurun_out/fp.log; exit 1; }
grep "us per link" gpurun_out/fp.log
done
