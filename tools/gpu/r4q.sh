# k = 16 fused update + projection on 16x16x4 MFMA (k_nn_tn_m16): per-L timing against the earlier
# forms, the k = 16 solver tests, then the k = 16 bench line with it on and off
source ./tools/gpu/step.sh
MIGMRES_NT_M16=0 step 200 r4q_mb_old.txt ./tools/mb_k16
MIGMRES_NT_M16=2 step 200 r4q_mb_m16.txt ./tools/mb_k16
grep "k=16" gpurun_out/r4q_mb_m16.txt
step 300 r4q_tests.log python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_solver.py -m gpu -x -q --timeout 200 --timeout-method thread
grep -E "passed|failed" gpurun_out/r4q_tests.log | tail -1
VAR=MIGMRES_NT_M16 VALUES="1 0 1 0" ARGS="--k 16 --no-csr-spmm" STEPS=25 TAG=r4q_k16 bash tools/gpu/sweep.sh || exit 1
