# Round-4 session e: fixed tests, bsr3 two-lane variant (bit-exact tests + A/B), chunk-order
# knobs with the 576-row pad (A B A B for the box's run-to-run spread)
source ./tools/gpu/step.sh
export TMPDIR=/tmp
step 600 r4e_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py tests/test_gpu_chebyshev.py tests/test_gpu_formats.py
tail -3 gpurun_out/r4e_tests.log
MIGMRES_BSR3_H=2 step 300 r4e_bsr3h_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k bsr3 tests/test_gpu_configs.py::test_flan_proxy_spmm_bit_exact
tail -3 gpurun_out/r4e_bsr3h_tests.log
VAR=MIGMRES_BSR3_H VALUES="1 2 1 2" ARGS="--matrix FlanProxy --k 4 --no-csr-spmm" TAG=r4e_h bash tools/gpu/sweep.sh > /dev/null || exit 1
VAR=MIGMRES_BSR3_H VALUES="1 2" ARGS="--matrix FlanProxy --k 8 --no-csr-spmm" TAG=r4e_h8 bash tools/gpu/sweep.sh > /dev/null || exit 1
VAR=MIGMRES_TN_CONTIG VALUES="0 1 0 1" ARGS="--nx 128 --no-csr-spmm" TAG=r4e_tn128 bash tools/gpu/sweep.sh > /dev/null || exit 1
VAR=MIGMRES_NNG_CONTIG VALUES="0 1 0 1" ARGS="--nx 128 --no-csr-spmm" TAG=r4e_nng128 bash tools/gpu/sweep.sh > /dev/null || exit 1
VAR=MIGMRES_TN_CONTIG VALUES="0 1 0 1" ARGS="--no-csr-spmm" TAG=r4e_tn256 bash tools/gpu/sweep.sh > /dev/null || exit 1
VAR=MIGMRES_NNG_CONTIG VALUES="0 1 0 1" ARGS="--no-csr-spmm" TAG=r4e_nng256 bash tools/gpu/sweep.sh > /dev/null || exit 1
cat gpurun_out/sweep_r4e_*.txt
