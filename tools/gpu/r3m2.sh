# 7-point plane march (k_spmm_march7): parity tests, SpMM timing over prefetch depth, benches
source ./tools/gpu/step.sh
P=${PROF:-r3m2}
step 600 tests_$P.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "march or tpl3 or choice or spmm_bit"
step 600 tests2_$P.log python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_loopback.py tests/test_gpu_prec.py -k "march or fused or distributed_spmm"
MIGMRES_NO_MARCH=1 step 120 ts_tpl_$P.log python tools/time_spmm.py Laplace3D 256 8
for pd in 1 2 3 4; do
  MIGMRES_MARCH_PD=$pd step 120 ts_pd${pd}_$P.log python tools/time_spmm.py Laplace3D 256 8
done
MIGMRES_MARCH_SZ=32 step 120 ts_sz32_$P.log python tools/time_spmm.py Laplace3D 256 8
MIGMRES_MARCH_SZ=64 step 120 ts_sz64_$P.log python tools/time_spmm.py Laplace3D 256 8
step 120 ts_128_$P.log python tools/time_spmm.py Laplace3D 128 8
MIGMRES_NO_MARCH=1 step 120 ts_128tpl_$P.log python tools/time_spmm.py Laplace3D 128 8
step 300 bench_256_$P.json python bench.py --no-cpu-baseline
MIGMRES_NO_MARCH=1 step 300 bench_256_nomarch_$P.json python bench.py --no-cpu-baseline
grep -h "Laplace3D" gpurun_out/ts_*_$P.log
for f in 256 256_nomarch; do tail -1 gpurun_out/bench_${f}_$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value'],2), d['kernels'].get('spmm'))"; done
