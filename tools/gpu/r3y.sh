source ./tools/gpu/step.sh
P=${PROF:-r3y}
step 900 tests_relax_$P.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_relaxation.py tests/test_gpu_prec.py tests/test_gpu_known_answers.py tests/test_gpu_chebyshev.py tests/test_gpu_kernels.py -k "not tpl3_27"
