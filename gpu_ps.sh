source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-ps1}
step 600 pytest_ps_$P.log python -u -m pytest tests/test_gpu_pseudo.py tests/test_gpu_solver.py tests/test_gpu_orthomanager.py -m gpu -x -q --timeout 300 --timeout-method thread
step 300 bench_pseudo_$P.json python bench.py --no-cpu-baseline --solver GMRES --steps 50 --warmup 10
