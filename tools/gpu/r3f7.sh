# march7 with the fixed 7-point slot pattern: parity + timing + SALU count
source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3f7}
step 300 tests_$P.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_prec.py tests/test_gpu_loopback.py -k "march or fused or spmm_bit"
step 120 ts_256_$P.log python tools/time_spmm.py Laplace3D 256 8
step 120 ts_128_$P.log python tools/time_spmm.py Laplace3D 128 8
step 120 ts_jac_$P.log python tools/time_spmm.py Laplace3D 256 8 jacobi
step 90 pmc_sq_$P.log timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU -T --output-format csv -d gpurun_out/pmc_sq_$P -o run --kernel-include-regex "march7" -- python3 tools/time_spmm.py Laplace3D 256 8 x 10
step 300 bench_$P.json python bench.py --no-cpu-baseline
for f in gpurun_out/ts_*_$P.log; do echo "$(basename $f .log): $(grep Laplace3D $f)"; done
tail -1 gpurun_out/bench_$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', round(d['value'],2), d['kernels'].get('spmm'))"
