source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3f}
step 200 pytest_tpl_$P.log python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "tpl3 or kernel_choice"
T="python tools/time_spmm.py"
step 120 ts_b_$P.log $T Brick3D 256 8
MIGMRES_TPL3_SHORT=1 step 120 ts_l7g_$P.log $T Laplace3D 256 8
MIGMRES_TPL3_SHORT=1 MIGMRES_TPL3_KC=8 step 120 ts_l7g8_$P.log $T Laplace3D 256 8
MIGMRES_TPL3_SHORT=1 MIGMRES_TPL3_KC=8 MIGMRES_TPL3_SLABS=0 step 120 ts_l7g80_$P.log $T Laplace3D 256 8
MIGMRES_TPL3_SHORT=1 MIGMRES_TPL3_SLABS=0 step 120 ts_l7g40_$P.log $T Laplace3D 256 8
step 120 ts_l7_$P.log $T Laplace3D 256 8
