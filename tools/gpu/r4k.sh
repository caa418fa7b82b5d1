# Round-4 session k: pair kernel without scale registers -- kernel tests + CSR forms
source ./tools/gpu/step.sh
export TMPDIR=/tmp
step 300 r4k_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_prec.py tests/test_gpu_loopback.py
tail -3 gpurun_out/r4k_tests.log
for i in 1 2; do
  step 300 r4k_b$i.json python bench.py --no-cpu-baseline --steps 25 --warmup 25 || exit 1
  python3 -c "
import json
l=[x for x in open('gpurun_out/r4k_b$i.json') if x.startswith('{')][-1]
d=json.loads(l); r=d['roofline_spmm']
print('run $i', round(d['value'],2), 'march', round(r['mean_launch_us'],1), {k:(round(v['mean_launch_us'],1), round(v['frac'],3)) for k,v in r['csr_forms'].items()})"
done
