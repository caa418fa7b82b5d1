# march7 lines per thread x prefetch depth: parity, SpMM timing sweep, benches
source ./tools/gpu/step.sh
P=${PROF:-r3m4}
step 600 tests_$P.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_prec.py tests/test_gpu_loopback.py -k "march or fused or distributed_spmm or spmm_bit"
for nl in 1 2; do for pd in 1 2 3; do
  MIGMRES_MARCH_NL=$nl MIGMRES_MARCH_PD=$pd step 120 ts_256_nl${nl}pd${pd}_$P.log python tools/time_spmm.py Laplace3D 256 8
  MIGMRES_MARCH_NL=$nl MIGMRES_MARCH_PD=$pd step 120 ts_128_nl${nl}pd${pd}_$P.log python tools/time_spmm.py Laplace3D 128 8
done; done
MIGMRES_MARCH_NL=2 MIGMRES_MARCH_SZ=128 step 120 ts_256_nl2sz128_$P.log python tools/time_spmm.py Laplace3D 256 8
step 120 ts_256_jac_$P.log python tools/time_spmm.py Laplace3D 256 8 jacobi
for f in gpurun_out/ts_*_$P.log; do echo "$(basename $f .log): $(grep Laplace3D $f)"; done
