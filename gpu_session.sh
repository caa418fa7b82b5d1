source ./tools_gpu_check.sh
step 120 mb_gemm_tn.log ./tools/mb_gemm_tn
step 600 t_solver.log python -m pytest tests/test_gpu_solver.py -q
