set -e
for v in w4 w5 w6 w7; do RTPT_LIB=variants/librtpt_$v.so timeout -k 10 200 python bench.py --scene spheres --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/sph_$v.log 2>&1; done
