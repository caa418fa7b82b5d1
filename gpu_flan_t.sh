source ./tools_gpu_check.sh
export TMPDIR=/tmp
step 300 pytest_flan_t.log python -u -m pytest tests/test_gpu_configs.py -m gpu -q --timeout 300 --timeout-method thread -k "flan_proxy_spmm" --tb=line -p no:warnings
