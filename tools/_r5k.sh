set -u
cd $GRAFT_REPO_ROOT
true
AB_K="headline or clusters or boxes or quads or golden" bash tools/ab.sh r5k base cluhelp cluhelp6 || exit 1
AB_NOTEST=1 bash tools/ab.sh r5k notrace || exit 1
for v in stats cluhelpst; do
  RTPT_LIB=$PWD/abvar/librtpt_$v.so timeout -k 10 200 python tools/kernel_stats.py 1920 1080 64 > gpurun_out/r5k/kstats_$v.json 2> gpurun_out/r5k/kstats_$v.err || { tail -5 gpurun_out/r5k/kstats_$v.err >&2; exit 1; }
done
# tail-effect diagnostic: the same 530.8 M samples as 3840x2160 x 64 spp
for w in lockstep free; do
  RTPT_WALK=$w timeout -k 10 200 python bench.py --scene spheres --width 3840 --height 2160 --spp 64 --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/r5k/sph4k_$w.json 2> gpurun_out/r5k/sph4k_$w.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/r5k/sph4k_$w.json sph4k_$w >&2
done
AB_NOTEST=1 bash tools/ab_mis_run.sh r5k base mis8 mis6
NOTEST=1 bash tools/r5_ab.sh r5k tri100k tri1m || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "triangle_bvh or c_abi or mis_lds" > gpurun_out/r5k/tri_tests.log 2>&1; tail -3 gpurun_out/r5k/tri_tests.log >&2
