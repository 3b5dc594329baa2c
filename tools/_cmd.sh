set -e
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k progressive > gpurun_out/tests.log 2>&1
timeout -k 10 400 python bench.py --width 8192 --height 8192 --spp 512 --batch-spp 64 --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/c5.log 2>&1
timeout -k 10 400 python bench.py --width 4096 --height 4096 --spp 128 --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/c3.log 2>&1
