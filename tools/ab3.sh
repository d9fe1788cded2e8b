#!/bin/bash
# A/B/C of bench variants in one GPU session: "<label>:<env assignments>" arguments, alternating, one
# JSON summary line each (extra bench.py flags from $BENCH_ARGS).  usage: bash tools/ab3.sh rounds "base:" "s16:AVT_LIB_PATH=..." ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
N=$1; shift
for i in $(seq 1 $N); do
  for spec in "$@"; do
    label=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab3.log 2>&1 || { tail -5 gpurun_out/ab3.log; exit 1; }
    python - "$label" <<'PY'
import json, sys
r = json.loads(open("gpurun_out/ab3.log").read().strip().splitlines()[-1])
k = r["roofline"]["per_kind"]
print(f"{sys.argv[1]:14s} {r['value']:9.1f} clips/s  {r['ms_per_step']:7.3f} ms  conv " +
      "  ".join(f"{n} {v['tflops']:.0f}/{v['ms_per_step']:.2f}ms" for n, v in k.items()), flush=True)
PY
  done
done
