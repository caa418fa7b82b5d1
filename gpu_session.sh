source ./tools_gpu_check.sh
step 300 tsolve.log python tools/time_solve.py 256
