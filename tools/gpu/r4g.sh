# Round-4 session g: full GPU suite, then the k x k steps in the pass prologues (FBG_PRO) A/B
source ./tools/gpu/step.sh
export TMPDIR=/tmp
rm -f gpurun_out/parity_margins.jsonl
step 900 pytest_gpu_r4g.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
cp gpurun_out/parity_margins.jsonl gpurun_out/parity_margins_r4g.jsonl
tail -3 gpurun_out/pytest_gpu_r4g.log
MIGMRES_FORCE_RCCL=1 VAR=MIGMRES_FBG_PRO VALUES="0 1 0 1" ARGS="--nx 128 --no-csr-spmm" TAG=r4g_pro128 bash tools/gpu/sweep.sh > /dev/null || exit 1
VAR=MIGMRES_FBG_PRO VALUES="0 1 0 1" ARGS="--no-csr-spmm" TAG=r4g_pro256 bash tools/gpu/sweep.sh > /dev/null || exit 1
VAR=MIGMRES_FBG_PRO VALUES="0 1" ARGS="--no-csr-spmm --ortho DGKS" TAG=r4g_dgks bash tools/gpu/sweep.sh > /dev/null || exit 1
cat gpurun_out/sweep_r4g_*.txt
MIGMRES_FORCE_RCCL=1 TAG=r4g_rccl128 ARGS="--nx 128 --no-csr-spmm" bash tools/gpu/trace.sh > /dev/null || exit 1
head -24 gpurun_out/timeline_r4g_rccl128.txt
