source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-k16c}
step 600 pytest_k16_$P.log python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "k16 or solves"
step 300 bench_k16_$P.log python bench.py --no-cpu-baseline --k 16
