source ./tools_gpu_check.sh
export TMPDIR=/tmp
step 1100 pytest_all.log python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread --durations=25
