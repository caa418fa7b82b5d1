source ./tools_gpu_check.sh
export TMPDIR=/tmp
step 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 600 bench.log python bench.py
