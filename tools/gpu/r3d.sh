# tpl3 walk-order / column-chunk sweep (SpMM device time) + tpl3 tests
source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3d}
step 200 pytest_tpl3_$P.log python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "tpl3"
T="python tools/time_spmm.py"
step 120 ts_$P.log $T Brick3D 256 8
MIGMRES_TPL3_SLABS=1 step 120 ts_slabs_$P.log $T Brick3D 256 8
MIGMRES_TPL3_KC=4 step 120 ts_kc4_$P.log $T Brick3D 256 8
MIGMRES_TPL3_KC=4 MIGMRES_TPL3_SLABS=1 step 120 ts_kc4s_$P.log $T Brick3D 256 8
MIGMRES_NO_TPL3=1 step 120 ts_notpl3_$P.log $T Brick3D 256 8
step 120 ts_l7_$P.log $T Laplace3D 256 8
step 120 ts_b384_$P.log $T Brick3D 384 8 x 10
MIGMRES_TPL3_SLABS=1 step 120 ts_b384s_$P.log $T Brick3D 384 8 x 10
