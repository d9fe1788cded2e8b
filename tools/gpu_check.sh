#!/bin/bash
# One GPU-box session: the steps given as arguments, in order.  Every GPU step runs under its own time
# limit; a failing step ends the session (no further GPU work after a crash, abort or timeout).
#   tests                  full GPU parity suite (stops at the first failure; MAXFAIL=n for more), then smoke()
#   t:<pytest args>        a subset of the GPU tests, e.g. "t:tests/test_kernels_gpu.py -k 'halo or c64'" (eval'd)
#   bench:<tag>:<args>     python bench.py <args>  -> gpurun_out/bench_<tag>.log (last line = the JSON)
#   prof:<tag>:<args>      rocprofv3 --kernel-trace --stats over bench.py --steps 5 --warmup 2 <args>
#                          -> gpurun_out/prof_<tag>/ and gpurun_out/kstats_<tag>.txt (per-step kernel table)
#   conv:<tag>:<args>      python tools/conv_bench.py <args> -> gpurun_out/conv_<tag>.log
#   ab:<rounds>:<spec>|<spec>...   tools/ab3.sh (same-box A/B; BENCH_ARGS from the environment)
# usage: bash tools/gpu_check.sh tests "bench:b128:" "bench:b32:--batch 32 --traffic-out gpurun_out/t32.json"
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  kind=${step%%:*}; rest=${step#*:}
  case "$kind" in
    tests)
      timeout -k 10 900 python -u -m pytest tests --maxfail=${MAXFAIL:-1} -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/gpu_tests.log 2>&1; rc=$?
      echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_tests.log | tail -8
      [ $rc -ne 0 ] && exit $rc
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
      echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
      [ $rc -ne 0 ] && exit $rc ;;
    t)
      eval "timeout -k 10 600 python -u -m pytest $rest -x -q -m gpu --timeout 300 --timeout-method thread \
        -p no:cacheprovider" > gpurun_out/gpu_t.log 2>&1; rc=$?
      echo "t rc=$rc ($rest)"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/gpu_t.log | tail -8
      [ $rc -ne 0 ] && exit $rc ;;
    bench)
      tag=${rest%%:*}; args=${rest#*:}
      timeout -k 10 600 python bench.py $args > gpurun_out/bench_$tag.log 2>&1; rc=$?
      echo "bench $tag rc=$rc"; tail -1 gpurun_out/bench_$tag.log | cut -c1-600
      [ $rc -ne 0 ] && exit $rc ;;
    prof)
      tag=${rest%%:*}; args=${rest#*:}
      rm -rf gpurun_out/prof_$tag
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$tag" -o run -- \
        python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --traffic off --no-peaks $args \
        > gpurun_out/prof_$tag.log 2>&1; rc=$?
      echo "prof $tag rc=$rc"; tail -1 gpurun_out/prof_$tag.log | cut -c1-300
      [ $rc -ne 0 ] && exit $rc
      python tools/kstats.py gpurun_out/prof_$tag/run_kernel_stats.csv auto 60 > gpurun_out/kstats_$tag.txt ;;
    conv)
      tag=${rest%%:*}; args=${rest#*:}
      timeout -k 10 400 python tools/conv_bench.py $args > gpurun_out/conv_$tag.log 2>&1; rc=$?
      echo "conv $tag rc=$rc"; grep -v amdgpu.ids gpurun_out/conv_$tag.log | tail -40
      [ $rc -ne 0 ] && exit $rc ;;
    ab)
      n=${rest%%:*}; specs=${rest#*:}
      IFS='|' read -ra S <<< "$specs"
      bash tools/ab3.sh "$n" "${S[@]}"; rc=$?
      [ $rc -ne 0 ] && exit $rc ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
