source ./tools/gpu/step.sh
P=${PROF:-r3final}
step 300 bench_k16_$P.json python bench.py --no-cpu-baseline --k 16
step 300 bench_bj_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
step 300 bench_flan_$P.json python bench.py --no-cpu-baseline --matrix FlanProxy --k 4
step 300 bench_dgks_$P.json python bench.py --no-cpu-baseline --ortho DGKS
for f in k16 bj flan dgks; do tail -1 gpurun_out/bench_${f}_$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value'],2), d['roofline']['kernel'], round(d['roofline']['frac'],3))"; done
