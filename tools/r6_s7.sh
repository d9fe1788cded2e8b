#!/bin/bash
# round-6 session 7: re-measure the BN-backward reductions fused into the dgrad epilogues (AVT_FUSE_BN_BWD=1; round 2-3:
# -1 %) now that removing the separate reductions is worth up to 3.4 % (B=128) / 4.3 % (B=32) (profiles/r6_bn_skip.txt)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export BENCH_ARGS="--traffic off --no-peaks --steps 20 --warmup 5"
bash tools/ab3.sh 3 "sep:AVT_FUSE_BN_BWD=0" "fused:AVT_FUSE_BN_BWD=1" > gpurun_out/ab_fuse_b128.log 2>&1 || { tail -5 gpurun_out/ab_fuse_b128.log; exit 1; }
cat gpurun_out/ab_fuse_b128.log
export BENCH_ARGS="--traffic off --no-peaks --steps 30 --warmup 5 --batch 32"
bash tools/ab3.sh 3 "sep:AVT_FUSE_BN_BWD=0" "fused:AVT_FUSE_BN_BWD=1" > gpurun_out/ab_fuse_b32.log 2>&1 || { tail -5 gpurun_out/ab_fuse_b32.log; exit 1; }
cat gpurun_out/ab_fuse_b32.log
echo ALL_OK
# upper bound of folding the wgrad slab reduces into the wgrad kernels (AVT_DIAG_SKIP 4: the reduce launches left out
# of the captured step; the gradient buffer is persistent and zeroed each step, so every tensor stays realistic)
: > gpurun_out/slabskip.log
for round in 1 2; do
  for B in 128 32; do
    for skip in 0 4; do
      timeout -k 10 200 env AVT_LIB_PATH="$R/audio-visual-tubes_amd/libavt_diag.so" AVT_DIAG_SKIP=$skip \
        python tools/step_time.py --batch $B --steps 20 --warmup 5 > gpurun_out/st.log 2>&1 || { tail -5 gpurun_out/st.log; exit 1; }
      tail -1 gpurun_out/st.log | tee -a gpurun_out/slabskip.log
    done
  done
done
echo ALL_OK2
