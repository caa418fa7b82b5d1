source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-xr1}
step 1000 pytest_gpu_$P.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 300 bench_flan_$P.json python bench.py --no-cpu-baseline --matrix FlanProxy --k 4
MIGMRES_NO_SELL_XR=1 step 300 bench_flan_${P}_off.json python bench.py --no-cpu-baseline --matrix FlanProxy --k 4
MIGMRES_NO_TPL_SPMM=1 step 300 bench_brick_sell_$P.json python bench.py --no-cpu-baseline --matrix Brick3D
