#!/bin/bash
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/pmc_c64.sh || exit 1
bash tools/ab3.sh 3 "c64on:AVT_C64=1" "c64off:AVT_C64=0"
