#!/bin/bash
# round-6 session 6 (measure first): the upper bound of removing the BN backward reductions
# (AVT_DIAG_SKIP 8) and the forward BN applies (16) from the captured step -- -DAVT_DIAG build (libavt_diag.so),
# WRONG results, the replays run on the eager warm-up's statistics and tensors (realistic data); tools/step_time.py,
# alternating, B=128 and B=32
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
: > gpurun_out/bnskip.log
for round in 1 2; do
  for B in 128 32; do
    for skip in 0 8 16 24; do
      timeout -k 10 200 env AVT_LIB_PATH="$R/audio-visual-tubes_amd/libavt_diag.so" AVT_DIAG_SKIP=$skip \
        python tools/step_time.py --batch $B --steps 20 --warmup 5 > gpurun_out/st.log 2>&1 || { tail -5 gpurun_out/st.log; exit 1; }
      tail -1 gpurun_out/st.log | tee -a gpurun_out/bnskip.log
    done
  done
done
echo ALL_OK
