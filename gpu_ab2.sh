source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-ab2}
step 600 pytest_kern_$P.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solver.py -m gpu -x -q --timeout 300 --timeout-method thread
B="python bench.py --no-cpu-baseline"
step 300 ab_nb8a_$P.json $B
step 300 ab_nb16a_$P.json env MIGMRES_NNG_NB=16 $B
step 300 ab_nb8b_$P.json $B
step 300 ab_nb16b_$P.json env MIGMRES_NNG_NB=16 $B
