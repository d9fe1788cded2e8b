#!/bin/bash
# A/B of two in-tree builds of libavt on the bench workload: alternating runs, one line each.
# usage: bash tools/ab_bench.sh <libA.so> <libB.so> [rounds] [bench args...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
A=$1; B=$2; N=${3:-2}; shift 3
for i in $(seq 1 $N); do
  for L in $A $B; do
    AVT_LIB_PATH=$R/audio-visual-tubes_amd/$L timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python - "$L" <<'PY'
import json, sys
r = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = r["roofline"]["per_kind"]
print(f"{sys.argv[1]:18s} {r['value']:9.1f} clips/s  {r['ms_per_step']:7.3f} ms  conv " +
      "  ".join(f"{n} {v['tflops']:.0f}" for n, v in k.items()))
PY
  done
done
