source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-xr2}
step 300 bench_flan8_$P.json python bench.py --no-cpu-baseline --matrix FlanProxy --k 8 --no-profile
MIGMRES_NO_SELL_XR=1 step 300 bench_flan8_${P}_off.json python bench.py --no-cpu-baseline --matrix FlanProxy --k 8 --no-profile
MIGMRES_NO_TPL_SPMM=1 step 300 bench_brick4_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --k 4
MIGMRES_NO_TPL_SPMM=1 MIGMRES_NO_SELL_XR=1 step 300 bench_brick4_${P}_off.json python bench.py --no-cpu-baseline --matrix Brick3D --k 4
MIGMRES_NO_TPL_SPMM=1 MIGMRES_NO_SELL_XR=1 step 300 bench_brick8_${P}_off.json python bench.py --no-cpu-baseline --matrix Brick3D --k 8
