source ./tools/gpu/step.sh
P=${PROF:-r3zc}
step 900 tests_$P.log python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests
step 300 bench_128_$P.json python bench.py --no-cpu-baseline --nx 128
step 300 bench_256_$P.json python bench.py --no-cpu-baseline
tail -2 gpurun_out/tests_$P.log
for f in 128 256; do tail -1 gpurun_out/bench_${f}_$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value'],2), d['kernels']['reduce'])"; done
