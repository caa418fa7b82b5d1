# Round-4 session j: the CSR SpMM forms (roofline_spmm.csr_forms) against the leading-dimension pad
source ./tools/gpu/step.sh
export TMPDIR=/tmp
for pad in 64 576 64 576; do
  MIGMRES_LD_PAD=$pad step 300 r4j_pad$pad.json python bench.py --no-cpu-baseline --steps 25 --warmup 25 || exit 1
  python3 -c "
import json,sys
l=[x for x in open('gpurun_out/r4j_pad$pad.json') if x.startswith('{')][-1]
d=json.loads(l); r=d['roofline_spmm']
print('pad $pad', round(d['value'],2), 'march', round(r['mean_launch_us'],1), {k:(round(v['mean_launch_us'],1), round(v['frac'],3)) for k,v in r['csr_forms'].items()})"
done
