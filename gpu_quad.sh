source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-q1}
step 900 pytest_quad_$P.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prec.py tests/test_gpu_configs.py tests/test_gpu_loopback.py -m gpu -x -q --timeout 300 --timeout-method thread
step 300 bench_bj_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
MIGMRES_NO_TPL_QUAD=1 step 300 bench_bj_${P}_off.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
step 300 bench_b_$P.json python bench.py --no-cpu-baseline --matrix Brick3D
