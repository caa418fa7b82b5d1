# march27 work items per CU (Brick3D + right Jacobi, 256^3); march7 WPC 1 vs 2 at 128^3
VAR=MIGMRES_MARCH27_WPC VALUES="9 2 4 9 2" ARGS="--matrix Brick3D --prec right --no-csr-spmm" TAG=r4p_bj bash tools/gpu/sweep.sh || exit 1
export MIGMRES_FORCE_RCCL=1
VAR=MIGMRES_MARCH_WPC VALUES="2 1 2 1" ARGS="--nx 128 --no-csr-spmm" TAG=r4p_128 bash tools/gpu/sweep.sh || exit 1
