# march7 work items per CU (slab size) at 256^3 and the per-rank shapes; march tests
source ./tools/gpu/step.sh
step 300 r4n_tests.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_loopback.py -m gpu -x -q --timeout 120 --timeout-method thread
VAR=MIGMRES_MARCH_WPC VALUES="2 9 4 2 9" ARGS="--no-csr-spmm" TAG=r4n_256 bash tools/gpu/sweep.sh || exit 1
export MIGMRES_FORCE_RCCL=1
VAR=MIGMRES_MARCH_WPC VALUES="2 9 2 9" ARGS="--nx 128 --no-csr-spmm" TAG=r4n_128 bash tools/gpu/sweep.sh || exit 1
VAR=MIGMRES_MARCH_WPC VALUES="2 9 2 9" ARGS="--nz 32 --no-csr-spmm" TAG=r4n_nz32 bash tools/gpu/sweep.sh || exit 1
