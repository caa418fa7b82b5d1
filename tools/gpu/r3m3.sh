# march7 with one column per workgroup: parity, SpMM timing over slab size and prefetch, benches
source ./tools/gpu/step.sh
P=${PROF:-r3m3}
step 600 tests_$P.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_prec.py tests/test_gpu_loopback.py -k "march or fused or distributed_spmm or spmm_bit"
for sz in 0 16 32 64 128; do
  MIGMRES_MARCH_SZ=$sz step 120 ts_256_sz${sz}_$P.log python tools/time_spmm.py Laplace3D 256 8
done
MIGMRES_MARCH_PD=3 step 120 ts_256_pd3_$P.log python tools/time_spmm.py Laplace3D 256 8
MIGMRES_MARCH_PD=1 step 120 ts_256_pd1_$P.log python tools/time_spmm.py Laplace3D 256 8
for sz in 0 8 16 32; do
  MIGMRES_MARCH_SZ=$sz step 120 ts_128_sz${sz}_$P.log python tools/time_spmm.py Laplace3D 128 8
done
MIGMRES_NO_MARCH=1 step 120 ts_128_tpl_$P.log python tools/time_spmm.py Laplace3D 128 8
step 300 bench_256_$P.json python bench.py --no-cpu-baseline
step 300 bench_128_$P.json python bench.py --no-cpu-baseline --nx 128
step 300 bench_k16_$P.json python bench.py --no-cpu-baseline --k 16
for f in gpurun_out/ts_*_$P.log; do echo "$(basename $f .log): $(grep Laplace3D $f)"; done
for f in 256 128 k16; do tail -1 gpurun_out/bench_${f}_$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value'],2), d['kernels'].get('spmm'))"; done
