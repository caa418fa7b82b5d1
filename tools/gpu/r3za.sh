source ./tools/gpu/step.sh
P=${PROF:-r3za}
step 600 tests_cheb_$P.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_chebyshev.py
step 400 bench_cheb_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right --prec-type chebyshev --cheb-degree 3
tail -1 gpurun_out/bench_cheb_$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cheb', d['value'], d['ms_per_step']); print({k:(round(v['ms'],1),v['launches']) for k,v in d['kernels'].items()})"
