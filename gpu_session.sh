source ./tools_gpu_check.sh
step 300 t_kernels.log python -m pytest tests/test_gpu_kernels.py -x -q
step 600 t_solver.log python -m pytest tests/test_gpu_solver.py -x -q
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step 600 bench.log python bench.py --steps 50 --warmup 5 --no-cpu-baseline
