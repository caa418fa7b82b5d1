# plane-march SpMM: parity tests, then SpMM timing march vs template kernels, then benches
source ./tools/gpu/step.sh
P=${PROF:-r3m1}
step 600 tests_$P.log python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "march or tpl3 or choice or spmm_bit"
step 600 tests2_$P.log python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_loopback.py tests/test_gpu_prec.py -k "march or fused or distributed_spmm"
for kind in Laplace3D Brick3D; do
  step 120 ts_${kind}_march_$P.log python tools/time_spmm.py $kind 256 8
  MIGMRES_NO_MARCH=1 step 120 ts_${kind}_tpl_$P.log python tools/time_spmm.py $kind 256 8
  MIGMRES_MARCH_KC=1 step 120 ts_${kind}_kc1_$P.log python tools/time_spmm.py $kind 256 8
  MIGMRES_MARCH_PD=2 step 120 ts_${kind}_pd2_$P.log python tools/time_spmm.py $kind 256 8
  MIGMRES_MARCH_PD=2 MIGMRES_MARCH_KC=1 step 120 ts_${kind}_pd2kc1_$P.log python tools/time_spmm.py $kind 256 8
done
step 300 bench_256_$P.json python bench.py --no-cpu-baseline
MIGMRES_NO_MARCH=1 step 300 bench_256_nomarch_$P.json python bench.py --no-cpu-baseline
step 300 bench_128_$P.json python bench.py --no-cpu-baseline --nx 128
step 300 bench_bj_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
grep -h "Laplace3D\|Brick3D" gpurun_out/ts_*_$P.log
for f in 256 256_nomarch 128 bj; do tail -1 gpurun_out/bench_${f}_$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value'],2), d['kernels'].get('spmm'))"; done
