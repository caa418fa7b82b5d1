# Secondary bench lines of a round (one per DESIGN section 7 row): PROF names the outputs.
source ./tools/gpu/step.sh
P=${PROF:-sec}
B="python bench.py --no-cpu-baseline"
step 300 bench_k16_$P.json $B --k 16 --no-csr-spmm
step 300 bench_bj_$P.json $B --matrix Brick3D --prec right --no-csr-spmm
step 300 bench_flan_$P.json $B --matrix FlanProxy --k 4
step 300 bench_dgks_$P.json $B --ortho DGKS --no-csr-spmm
step 300 bench_pseudo_$P.json $B --solver GMRES --no-csr-spmm
step 300 bench_cheb_$P.json $B --matrix Brick3D --prec right --prec-type chebyshev --no-csr-spmm
MIGMRES_FORCE_RCCL=1 step 300 bench_nz32_$P.json $B --nz 32 --no-csr-spmm
for f in k16 bj flan dgks pseudo cheb nz32; do python3 tools/bench_summary.py gpurun_out/bench_${f}_$P.json $f; done
