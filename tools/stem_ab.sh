#!/bin/bash
# A/B of the 7x7/s2 stem kernel (AVT_STEM=1) against the generic gather kernel (AVT_STEM=0) on the bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for i in 1 2; do
  for v in 0 1; do
    AVT_STEM=$v timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/stem_ab.log 2>&1 || { tail -5 gpurun_out/stem_ab.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
r = json.loads(open("gpurun_out/stem_ab.log").read().strip().splitlines()[-1])
k = r["roofline"]["per_kind"]
print(f"AVT_STEM={sys.argv[1]} {r['value']:9.1f} clips/s  {r['ms_per_step']:7.3f} ms  conv " +
      "  ".join(f"{n} {v['tflops']:.0f} {v['ms_per_step']:.3f}ms" for n, v in k.items()))
PY
  done
done
