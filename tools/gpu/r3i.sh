source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3i}
step 200 pytest_b3_$P.log python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "bsr3"
T="python tools/time_spmm.py"
step 120 ts_f4_$P.log $T FlanProxy 0 4
MIGMRES_BSR3_J=4 step 120 ts_f4j4_$P.log $T FlanProxy 0 4
MIGMRES_BSR3_J=1 step 120 ts_f4j1_$P.log $T FlanProxy 0 4
MIGMRES_BSR3_J=4 step 120 ts_f2j4_$P.log $T FlanProxy 0 2
step 120 ts_f2_$P.log $T FlanProxy 0 2
step 120 ts_f1_$P.log $T FlanProxy 0 1
