#!/bin/bash
# Round 3: what bounds the TN wgrad at B=32 (V.l3 / A.l4): AVT_TN_DBG bits 1 no memory, 2 no MFMA, 4 no epilogue stores, 8 no k loop
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd)
for S in "V.l3" "A.l4"; do
for d in 0 3 7 8 12 15; do
  rm -rf gpurun_out/tndbg
  AVT_TN_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/tndbg" -o run -- python "$R/tools/conv_bench.py" --batch 32 --only "$S" --kinds wgrad --variants 1 > gpurun_out/tndbg.log 2>&1 || { echo "dbg $d failed"; tail -3 gpurun_out/tndbg.log; exit 1; }
  python - "$R/gpurun_out/tndbg/run_kernel_stats.csv" "$S dbg=$d" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "conv_tn" in n or "reduce" in n:
        print(f"{sys.argv[2]:12s} {float(r['AverageNs'])/1e3:8.1f} us  {n[:50]}")
PY
done; done
