source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3g}
rm -f gpurun_out/parity_margins.jsonl
step 600 pytest_gpu_$P.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
cp gpurun_out/parity_margins.jsonl gpurun_out/parity_margins_$P.jsonl
step 300 bench_bj_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
step 300 bench_flan_$P.json python bench.py --no-cpu-baseline --matrix FlanProxy --k 4
step 300 bench_k16_$P.json python bench.py --no-cpu-baseline --k 16
