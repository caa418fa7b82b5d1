source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-k16d}
step 900 pytest_k16_$P.log python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_configs.py tests/test_gpu_loopback.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread
step 300 bench_k16_$P.json python bench.py --no-cpu-baseline --k 16 --steps 50 --warmup 26
