source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-s2}
step 300 pytest_kat_$P.log python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "known_answers"
step 300 bench_k16_$P.log python bench.py --no-cpu-baseline --k 16
step 300 bench_brickjac_$P.log python bench.py --no-cpu-baseline --matrix Brick3D --prec right --steps 50 --warmup 25
step 300 bench_brickjacf_$P.log python bench.py --no-cpu-baseline --matrix Brick3D --prec right --solver "FLEXIBLE GMRES" --steps 50 --warmup 25
