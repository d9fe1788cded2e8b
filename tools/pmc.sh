# PMC counter passes over the conv microbenchmark (one kernel shape), kernel-trace only.
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
if [ "$1" = list ]; then timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1; echo "list rc=$?"; grep -c . gpurun_out/pmc/counters.txt; exit 0; fi
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run -- python "$R/tools/conv_bench.py" $CB_ARGS > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
  echo "pass $i ok: $ctrs"
done
