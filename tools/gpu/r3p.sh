source ./tools/gpu/step.sh
P=${PROF:-r3p}
step 600 tests_cheb_$P.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_chebyshev.py
