#!/bin/bash
# round-6 session 19: the marginal cost of one BN finalize launch in the captured step -- the -DAVT_DIAG build with the
# forward (AVT_DIAG_SKIP 32) / backward (64) finalizes launched TWICE (a valid measurement: the duplicate writes the same
# scale/shift/k1/k2, every tensor keeps realistic values); tools/step_time.py, alternating, B=32 and B=128
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
: > gpurun_out/findup.log
for round in 1 2; do
  for B in 32 128; do
    for bits in 0 32 64 96; do
      timeout -k 10 200 env AVT_LIB_PATH="$R/audio-visual-tubes_amd/libavt_diag.so" AVT_DIAG_SKIP=$bits \
        python tools/step_time.py --batch $B --steps 30 --warmup 5 > gpurun_out/st.log 2>&1 || { tail -5 gpurun_out/st.log; exit 1; }
      tail -1 gpurun_out/st.log | tee -a gpurun_out/findup.log
    done
  done
done
echo ALL_OK
