#!/bin/bash
# Same-box A/B of whole source trees (each with its own Python and its own in-tree libavt.so, e.g. earlier rounds
# exported by `git archive <rev> | tar -x -C abtrees/<name>` and built with that tree's __graft_entry__.build()).
# Alternates "<label>:<tree dir>:<extra bench.py args>" specs for $1 rounds with the driver's bench command
# (--gpus 1 --steps 20 --warmup 5, plus $BENCH_ARGS), one summary line per run.
# usage: bash tools/abtree.sh 3 "head:.:--traffic off --no-peaks" "r2:abtrees/r2:"
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
N=$1; shift
for i in $(seq 1 $N); do
  for spec in "$@"; do
    label=${spec%%:*}; rest=${spec#*:}; dir=${rest%%:*}; extra=${rest#*:}
    ( cd "$dir" && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $extra $BENCH_ARGS ) \
      > gpurun_out/abtree.log 2>&1 || { tail -5 gpurun_out/abtree.log; exit 1; }
    python - "$label" <<'PY'
import json, sys
r = json.loads(open("gpurun_out/abtree.log").read().strip().splitlines()[-1])
k = r.get("roofline", {}).get("per_kind", {})
print(f"{sys.argv[1]:10s} {r['value']:9.1f} clips/s  {r['ms_per_step']:7.3f} ms  conv " +
      "  ".join(f"{n} {v['tflops']:.0f}/{v['ms_per_step']:.2f}ms" for n, v in k.items()), flush=True)
PY
  done
done
