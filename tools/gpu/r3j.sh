source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3j}
MIGMRES_NT_PW=1 step 200 mbk16_pw_$P.log ./tools/mb_k16
MIGMRES_NT_PW=0 step 200 mbk16_old_$P.log ./tools/mb_k16
step 400 pytest_k16_$P.log python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_solver.py tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread -k "k16 or gram or config_solves or gemm"
step 300 bench_k16_$P.json python bench.py --no-cpu-baseline --k 16
MIGMRES_NT_PW=0 step 300 bench_k16_old_$P.json python bench.py --no-cpu-baseline --k 16
