source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-fc}
step 600 pytest_fc_$P.log python -u -m pytest tests/test_gpu_fillcomplete.py -x -v --timeout 300 --timeout-method thread
