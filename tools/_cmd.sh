set -e
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/tests.log 2>&1
timeout -k 10 200 python bench.py --scene spheres --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/sph_oct.log 2>&1
