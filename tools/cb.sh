mkdir -p gpurun_out
timeout -k 10 240 python -m pytest tests/test_kernels_gpu.py -q -x -m gpu -p no:cacheprovider > gpurun_out/k.log 2>&1; rc=$?; tail -2 gpurun_out/k.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/conv_bench.py $CB_ARGS > gpurun_out/conv_bench.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/conv_bench.log; exit $rc
