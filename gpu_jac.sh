source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-jac}
step 600 pytest_jac_$P.log python -u -m pytest tests/test_gpu_prec.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread
step 300 bench_bj_$P.log python bench.py --no-cpu-baseline --matrix Brick3D --prec right --steps 50 --warmup 25
step 300 bench_bj_nofuse_$P.log env MIGMRES_NO_FUSED_JACOBI=1 python bench.py --no-cpu-baseline --matrix Brick3D --prec right --steps 50 --warmup 25
