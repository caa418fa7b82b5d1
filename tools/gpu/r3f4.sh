# 3x3-block SpMM with 16-byte value loads: parity (FlanProxy / bsr3 cases), SpMM timing, FlanProxy bench
source ./tools/gpu/step.sh
P=${PROF:-r3f4}
step 600 tests_$P.log python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_formats.py tests/test_gpu_loopback.py tests/test_gpu_fillcomplete.py -k "Flan or flan or bsr3 or unstructured or formats or fillcomplete"
step 120 ts_flan4_$P.log python tools/time_spmm.py FlanProxy 0 4
step 120 ts_flan8_$P.log python tools/time_spmm.py FlanProxy 0 8
step 300 bench_flan_$P.json python bench.py --no-cpu-baseline --matrix FlanProxy --k 4
for f in gpurun_out/ts_*_$P.log; do echo "$(basename $f .log): $(grep FlanProxy $f)"; done
tail -1 gpurun_out/bench_flan_$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('flan', round(d['value'],2), d['kernels'].get('spmm'))"
