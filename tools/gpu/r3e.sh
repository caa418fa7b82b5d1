# SpMM walk-order / column-chunk sweep, 7- and 27-point
source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3e}
step 200 pytest_tpl_$P.log python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "tpl3 or kernel_choice"
T="python tools/time_spmm.py"
step 120 ts_l7_$P.log $T Laplace3D 256 8
MIGMRES_TPL_SLABS=1 step 120 ts_l7s_$P.log $T Laplace3D 256 8
MIGMRES_TPL_SLABS=1 MIGMRES_TPL_KC=4 step 120 ts_l7s4_$P.log $T Laplace3D 256 8
MIGMRES_TPL_KC=4 step 120 ts_l74_$P.log $T Laplace3D 256 8
MIGMRES_TPL3_KC=2 MIGMRES_TPL3_SLABS=1 step 120 ts_kc2s_$P.log $T Brick3D 256 8
MIGMRES_TPL3_KC=4 MIGMRES_TPL3_SLABS=1 step 120 ts_kc4s_$P.log $T Brick3D 256 8
MIGMRES_TPL3_KC=4 MIGMRES_TPL3_SLABS=1 step 120 ts_b384kc4s_$P.log $T Brick3D 384 8 x 10
MIGMRES_TPL_SLABS=1 step 120 ts_l7s16_$P.log $T Laplace3D 256 16
step 120 ts_l716_$P.log $T Laplace3D 256 16
