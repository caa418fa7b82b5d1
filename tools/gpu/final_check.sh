source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r2k}
step 1000 pytest_gpu_$P.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 300 smoke_$P.log python -c "import __graft_entry__ as g; g.smoke()"
step 400 bench_$P.log python bench.py
step 300 bench_bj_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
step 300 bench_k16_$P.json python bench.py --no-cpu-baseline --k 16
step 300 bench_flan_$P.json python bench.py --no-cpu-baseline --matrix FlanProxy --k 4
