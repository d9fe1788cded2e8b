#!/bin/bash
# Round 3: where the B=32 wgrad time goes: kernel stats of the TN kernel vs its slab reduce; PMC of the TN kernel
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd)
rm -rf gpurun_out/wprof; mkdir -p gpurun_out/wprof
for S in "V.l3" "V.l1" "V.ds3" "A.l4"; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/wprof/$S" -o run -- python "$R/tools/conv_bench.py" --batch 32 --only "$S" --kinds wgrad --variants 1 > gpurun_out/wprof/$S.log 2>&1 || { echo "prof $S failed"; tail -3 gpurun_out/wprof/$S.log; exit 1; }
echo "== $S"; grep -v amdgpu gpurun_out/wprof/$S.log | tail -2 | head -1
python - "$R/gpurun_out/wprof/$S/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "conv" in n or "reduce" in n:
        print(f"  {float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4s}  {n[:90]}")
PY
done
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
C2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVES"
C3="GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
i=0
for C in "$C1" "$C2" "$C3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/wprof/pmc$i" -o run -- python "$R/tools/conv_bench.py" --batch 32 --only "V.l3" --kinds wgrad --variants 1 > gpurun_out/wprof/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 gpurun_out/wprof/pmc$i.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/wprof/pmc*/run_counter_collection.csv | grep -A25 "conv_tn\|slab_reduce" | head -60
