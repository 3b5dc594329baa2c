set -e
for l in 1 2 3 4 6 8; do RTPT_BVH_LEAF=$l timeout -k 10 200 python bench.py --scene spheres --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/sph_leaf$l.log 2>&1; done
