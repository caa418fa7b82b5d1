source ./tools/gpu/step.sh
MIGMRES_NW_MIN_L=16 step 200 r4u_mb_w16.txt ./tools/mb_k16
grep "k= 8 L=[ 0-9]\{3\} " gpurun_out/r4u_mb_w16.txt | head -8
step 600 r4u_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
grep -hE "passed|failed" gpurun_out/r4u_tests.log | tail -1
VAR=MIGMRES_BSR3_C VALUES="1 0" ARGS="--matrix FlanProxy --k 4" STEPS=400 TAG=r4u_flan4 bash tools/gpu/sweep.sh || exit 1
