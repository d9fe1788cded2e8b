mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_model_gpu.py -q -s -m gpu -p no:cacheprovider > gpurun_out/m.log 2>&1; rc=$?; echo "model rc=$rc"; tail -3 gpurun_out/m.log
