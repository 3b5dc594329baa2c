set -e
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/tests.log 2>&1
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/b_fused.log 2>&1
for v in nofuse fw7; do RTPT_LIB=variants/librtpt_$v.so timeout -k 10 200 python bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/b_$v.log 2>&1; done
