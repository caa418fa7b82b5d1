# bsr3 node-padded interleaved X: tests, then FlanProxy k = 4 / k = 8 A/B (NOPAD=1 is the old layout)
source ./tools/gpu/step.sh
step 400 r4o_tests.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_formats.py tests/test_gpu_prec.py tests/test_gpu_configs.py tests/test_gpu_loopback.py -m gpu -x -q --timeout 200 --timeout-method thread
grep -E "passed|failed" gpurun_out/r4o_tests.log | tail -1
VAR=MIGMRES_BSR3_NOPAD VALUES="0 1 0 1" ARGS="--matrix FlanProxy --k 4 --no-csr-spmm" STEPS=400 TAG=r4o_flan4 bash tools/gpu/sweep.sh || exit 1
VAR=MIGMRES_BSR3_NOPAD VALUES="0 1" ARGS="--matrix FlanProxy --k 8 --no-csr-spmm" STEPS=200 TAG=r4o_flan8 bash tools/gpu/sweep.sh || exit 1
