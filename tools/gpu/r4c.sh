# Round-4 A/B session: chunk order of the basis passes, bsr3 id prefetch, march template-id skip, bsr3 PMC
source ./tools/gpu/step.sh
VAR=MIGMRES_TN_CONTIG VALUES="0 1" ARGS="--nx 128 --no-csr-spmm" TAG=r4c_tn128 bash tools/gpu/sweep.sh > /dev/null || exit 1
VAR=MIGMRES_NNG_CONTIG VALUES="0 1" ARGS="--nx 128 --no-csr-spmm" TAG=r4c_nng128 bash tools/gpu/sweep.sh > /dev/null || exit 1
VAR=MIGMRES_TN_CONTIG VALUES="0 1" ARGS="--no-csr-spmm" TAG=r4c_tn256 bash tools/gpu/sweep.sh > /dev/null || exit 1
VAR=MIGMRES_MARCH7_TID VALUES="1 0" ARGS="--no-csr-spmm" TAG=r4c_tid256 bash tools/gpu/sweep.sh > /dev/null || exit 1
VAR=MIGMRES_BSR3_PF VALUES="0 1" ARGS="--matrix FlanProxy --k 4 --no-csr-spmm" TAG=r4c_pf bash tools/gpu/sweep.sh > /dev/null || exit 1
MIGMRES_BSR3_J=4 VAR=MIGMRES_BSR3_PF VALUES="0 1" ARGS="--matrix FlanProxy --k 4 --no-csr-spmm" TAG=r4c_pf4 bash tools/gpu/sweep.sh > /dev/null || exit 1
VAR=MIGMRES_TN_COR VALUES="0 1" ARGS="--nx 128 --no-csr-spmm" TAG=r4c_cor128 bash tools/gpu/sweep.sh > /dev/null || exit 1
VAR=MIGMRES_TN_COR VALUES="0 1" ARGS="--no-csr-spmm" TAG=r4c_cor256 bash tools/gpu/sweep.sh > /dev/null || exit 1
cat gpurun_out/sweep_r4c_*.txt
TAG=r4c_flan KRE="spmm_bsr3|interleave" ARGS="--matrix FlanProxy --k 4" bash tools/gpu/pmc_kernel.sh > /dev/null || exit 1
cat gpurun_out/pmc_r4c_flan.txt
