source ./tools_gpu_check.sh
export TMPDIR=/tmp
step 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step 600 bench.log python bench.py
