source ./tools/gpu/step.sh
step 600 r4v_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -hE "passed|failed" gpurun_out/r4v_tests.log | tail -1
VAR=MIGMRES_NW_MIN_L VALUES="16 64 16 64" ARGS="--no-csr-spmm" TAG=r4v_256 bash tools/gpu/sweep.sh || exit 1
export MIGMRES_FORCE_RCCL=1
VAR=MIGMRES_NW_MIN_L VALUES="16 64 16 64" ARGS="--nx 128 --no-csr-spmm" TAG=r4v_128 bash tools/gpu/sweep.sh || exit 1
unset MIGMRES_FORCE_RCCL
VAR=MIGMRES_NW_MIN_L VALUES="16 64 16 64" ARGS="--matrix FlanProxy --k 4 --no-csr-spmm" STEPS=400 TAG=r4v_flan bash tools/gpu/sweep.sh || exit 1
