source ./tools/gpu/step.sh
MIGMRES_NT_M16=1 step 200 r4t_mb_m1.txt ./tools/mb_k16
MIGMRES_NT_M16=3 step 200 r4t_mb_m3.txt ./tools/mb_k16
grep "k= 8 L=[ 0-9]\{3\} " gpurun_out/r4t_mb_m1.txt gpurun_out/r4t_mb_m3.txt | head -20
MIGMRES_BSR3_C=1 step 300 r4t_tests_c2.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_prec.py -k "bsr3 or flan or Flan" -m gpu -x -q --timeout 200 --timeout-method thread
MIGMRES_BSR3_C=1 MIGMRES_BSR3_J=1 step 300 r4t_tests_c1.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_prec.py -k "bsr3 or flan or Flan" -m gpu -x -q --timeout 200 --timeout-method thread
grep -hE "passed|failed" gpurun_out/r4t_tests_c2.log gpurun_out/r4t_tests_c1.log
VAR=MIGMRES_BSR3_C VALUES="0 1 0 1" ARGS="--matrix FlanProxy --k 4 --no-csr-spmm" STEPS=400 TAG=r4t_flan4 bash tools/gpu/sweep.sh || exit 1
export MIGMRES_BSR3_J=1
VAR=MIGMRES_BSR3_C VALUES="0 1" ARGS="--matrix FlanProxy --k 4 --no-csr-spmm" STEPS=400 TAG=r4t_flan4j1 bash tools/gpu/sweep.sh || exit 1
VAR=MIGMRES_BSR3_C VALUES="0 1" ARGS="--matrix FlanProxy --k 8 --no-csr-spmm" STEPS=200 TAG=r4t_flan8 bash tools/gpu/sweep.sh || exit 1
