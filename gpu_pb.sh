source ./tools_gpu_check.sh
export TMPDIR=/tmp
step 400 pytest_pb.log python -u -m pytest tests/test_gpu_pseudo.py tests/test_gpu_configs.py tests/test_gpu_solver.py -x -q --timeout 200 --timeout-method thread
step 200 bench_pb.log python bench.py --no-cpu-baseline --solver GMRES --steps 50 --warmup 25
step 200 bench_pb0.log env MIGMRES_PSEUDO_BATCHED=0 python bench.py --no-cpu-baseline --solver GMRES --steps 50 --warmup 25
