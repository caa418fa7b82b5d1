source ./tools/gpu/step.sh
P=${PROF:-r3q}
step 900 tests_formats_$P.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_formats.py tests/test_gpu_fillcomplete.py
