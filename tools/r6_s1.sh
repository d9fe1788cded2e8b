#!/bin/bash
# round-6 session 1: the 2-rank bench test + new GPU tests, smoke, halo s_setprio A/B, the halo issue/park split PMC
# pass, one default bench line.  Every GPU step under its own time limit; stop at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; }
# a test failure (rc 1) is not a GPU fault: record it and go on; anything else (timeout, abort, segfault) stops
soft() { local name=$1; shift; "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || { tail -20 "gpurun_out/$name.log"; exit $rc; }; [ $rc -eq 0 ] || tail -25 "gpurun_out/$name.log"; }
soft t_new timeout -k 10 480 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_bench_dist_gpu.py \
  "tests/test_ddp_gpu.py::test_side_stream_adam_ordering_without_host_sync" \
  "tests/test_model_gpu.py::test_eval_mode_input_gradient_refused" tests/test_twoview_gpu.py
step smoke timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()"
step halo_prio timeout -k 10 180 tools/halo_bench 128 3 20
export CB_ARGS="--only V.l3,V.l4,A.l4 --kinds fwd,dgrad --variants 1"
step pmc bash tools/pmc.sh "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
step bench timeout -k 10 300 python bench.py --traffic off
echo ALL_OK
