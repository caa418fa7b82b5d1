source ./tools_gpu_check.sh
B="python bench.py --no-cpu-baseline"
step 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 300 chol_new.json $B
step 300 chol_s128new.json $B --nx 128 --steps 200 --warmup 50
