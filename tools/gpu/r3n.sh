source ./tools/gpu/step.sh
P=${PROF:-r3n}
step 600 tests_resolve_$P.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_resolve.py tests/test_gpu_pseudo.py -k "resolve or pseudo_gmres_hb or orthogonalization or parameter_lists"
