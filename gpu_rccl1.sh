source ./tools_gpu_check.sh
export TMPDIR=/tmp
step 300 pytest_rccl1.log python -u -m pytest tests/test_gpu_solver.py -x -v --timeout 200 --timeout-method thread -k "one_rank_rccl"
step 200 bench_rccl1.log env MIGMRES_FORCE_RCCL=1 python bench.py --no-cpu-baseline --steps 50 --warmup 25
step 200 bench_rccl1_128.log env MIGMRES_FORCE_RCCL=1 python bench.py --no-cpu-baseline --nx 128
