source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-nt}
step 600 pytest_nt_$P.log python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_solver.py -x -q --timeout 300 --timeout-method thread -k "k16 or solves or match"
step 300 bench_k16_$P.log python bench.py --no-cpu-baseline --k 16
step 300 bench_$P.log python bench.py --no-cpu-baseline
