set -e
timeout -k 10 600 python -m pytest tests/test_gpu_mis.py -x -q > gpurun_out/tests.log 2>&1
timeout -k 10 300 python tools/bench_mis.py > gpurun_out/mis.log 2>&1
