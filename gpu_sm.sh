source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-sm1}
step 600 pytest_sm_$P.log python -u -m pytest tests/test_gpu_pseudo.py tests/test_gpu_kernels.py tests/test_abi_consumer.py -m gpu -x -q --timeout 300 --timeout-method thread
