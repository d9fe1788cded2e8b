#!/bin/bash
# Round 3: split-K + schedule tests, step A/B (split-K, wgrad streams, overlapped Adam) at B=32 and B=128,
# per-shape B=32 conv table, halo PMC passes
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_splitk_gpu.py tests/test_schedule_gpu.py tests/test_ddp_gpu.py -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_sched.log 2>&1; rc=$?
echo "new tests rc=$rc"; grep -E "passed|failed|Error|\{" gpurun_out/t_sched.log | tail -12; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--batch 32 --steps 30" bash tools/ab3.sh 2 "old:" "adam:AVT_ADAM_OVERLAP=1" "split:AVT_ADAM_OVERLAP=1 AVT_SPLITK=1" "sp256:AVT_ADAM_OVERLAP=1 AVT_SPLITK=1 AVT_SPLITK_BLOCKS=256" "sp1k:AVT_ADAM_OVERLAP=1 AVT_SPLITK=1 AVT_SPLITK_BLOCKS=1024" "ws2:AVT_ADAM_OVERLAP=1 AVT_SPLITK=1 AVT_WGRAD_STREAMS=2" "ws1:AVT_ADAM_OVERLAP=1 AVT_SPLITK=1 AVT_WGRAD_STREAMS=1" "fusebn:AVT_ADAM_OVERLAP=1 AVT_SPLITK=1 AVT_FUSE_BN_BWD=1" || exit 1
BENCH_ARGS="--steps 20" bash tools/ab3.sh 2 "old:" "new:AVT_ADAM_OVERLAP=1 AVT_SPLITK=1" "ws2:AVT_ADAM_OVERLAP=1 AVT_SPLITK=1 AVT_WGRAD_STREAMS=2" || exit 1
timeout -k 10 300 python tools/conv_bench.py --batch 32 --variants 1 > gpurun_out/cb32.txt 2>&1 || { tail -5 gpurun_out/cb32.txt; exit 1; }
grep -v amdgpu gpurun_out/cb32.txt
timeout -k 10 300 python tools/conv_bench.py --batch 32 --only "3x3" --kinds none --variants 1 --splitk "1,2,4,8" > gpurun_out/cbsk32.txt 2>&1 || { tail -5 gpurun_out/cbsk32.txt; exit 1; }
grep -v amdgpu gpurun_out/cbsk32.txt
timeout -k 10 300 python tools/conv_bench.py --batch 128 --only "3x3" --kinds none --variants 1 --stages "2,3;3,3;4,3;5,3" > gpurun_out/cbst128.txt 2>&1 || { tail -5 gpurun_out/cbst128.txt; exit 1; }
grep -v amdgpu gpurun_out/cbst128.txt
# PMC stall breakdown of the layer4 halo kernels (B=128 shapes, fwd + dgrad): verdict r2 item 4
R=$(pwd); mkdir -p gpurun_out/pmc
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
C2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVES"
C3="GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for C in "$C1" "$C2" "$C3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/halo_p$i" -o run -- python "$R/tools/conv_bench.py" --only "l4 3x3" --kinds fwd,dgrad --variants 1 > gpurun_out/pmc/halo_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 gpurun_out/pmc/halo_p$i.log; exit 1; }
  echo "pmc pass $i ok"
done
