#!/bin/bash
# round-6 session 18: kernel traces of the graph-replayed step (no eager profiling steps) at B=32 and B=128, to read
# the GPU's idle time inside a replayed step (tools/timeline.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for B in 32 128; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/tl_b$B" -o run -- python3 "$R/bench.py" --batch $B --steps 20 --warmup 5 --prof-steps 0 --traffic off --no-peaks --no-cpu-baseline > "$R/gpurun_out/tl_b$B.log" 2>&1 || { echo "trace b$B failed"; tail -5 "$R/gpurun_out/tl_b$B.log"; exit 1; }
  echo "trace b$B ok"
done
echo ALL_OK
