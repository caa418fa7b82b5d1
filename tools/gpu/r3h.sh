source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3h}
step 300 pytest_b3_$P.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_loopback.py -x -v --timeout 120 --timeout-method thread -k "bsr3 or bit_exact or kernel_choice"
T="python tools/time_spmm.py"
step 120 ts_f4_$P.log $T FlanProxy 0 4
MIGMRES_NO_BSR3=1 step 120 ts_f4n_$P.log $T FlanProxy 0 4
step 120 ts_f8_$P.log $T FlanProxy 0 8
MIGMRES_NO_BSR3=1 step 120 ts_f8n_$P.log $T FlanProxy 0 8
step 300 bench_flan_$P.json python bench.py --no-cpu-baseline --matrix FlanProxy --k 4
