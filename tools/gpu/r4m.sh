# march slab size at the 8-GPU per-rank shapes (256x256x32 slab, 128^3), one-rank RCCL paths on
export MIGMRES_FORCE_RCCL=1
VAR=MIGMRES_MARCH_SZ VALUES="0 16 32 11 0" ARGS="--nz 32 --no-csr-spmm" TAG=r4m_nz32 bash tools/gpu/sweep.sh || exit 1
VAR=MIGMRES_MARCH_SZ VALUES="0 16 32 11 0" ARGS="--nx 128 --no-csr-spmm" TAG=r4m_128 bash tools/gpu/sweep.sh || exit 1
