source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-tpl}
step 600 pytest_tpl_$P.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_loopback.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread
step 300 bench_$P.log python bench.py --no-cpu-baseline
step 300 bench_brick_$P.log python bench.py --no-cpu-baseline --matrix Brick3D --steps 50 --warmup 25
step 300 bench_notpl_$P.log env MIGMRES_NO_TPL_SPMM=1 python bench.py --no-cpu-baseline
step 300 bench_brick_notpl_$P.log env MIGMRES_NO_TPL_SPMM=1 python bench.py --no-cpu-baseline --matrix Brick3D --steps 50 --warmup 25
