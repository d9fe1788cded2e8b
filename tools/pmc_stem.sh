# SQ counter passes over tools/stem_bench.py (the stem fwd/wgrad kernels), kernel-trace only; one
# rocprofv3 run per pass.  Usage: bash tools/pmc_stem.sh "CTR1 CTR2 ..." ["..."]  |  bash tools/pmc_stem.sh list
mkdir -p gpurun_out/pmc_stem
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
if [ "$1" = list ]; then timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_stem/counters.txt 2>&1; echo "list rc=$?"; exit 0; fi
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_stem/p$i" -o run -- python "$R/tools/stem_bench.py" > gpurun_out/pmc_stem/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_stem/p$i.log; exit 1; }
  echo "pass $i ok: $ctrs"
done
