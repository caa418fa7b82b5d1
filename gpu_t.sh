source ./tools_gpu_check.sh
export TMPDIR=/tmp
step 300 consumer.log timeout -k 10 200 tests/abi_consumer/mvop_tester
step 900 pytest_cfg.log python -u -m pytest tests/test_abi_consumer.py tests/test_gpu_configs.py tests/test_gpu_loopback.py tests/test_gpu_kernels.py -m gpu -v --timeout 400 --timeout-method thread
