# Round-4 session d: the new GPU tests, then the leading-dimension sweep at the per-rank sizes
# of the 1/2/4/8-GPU 256^3 runs (256 x 256 x nz), then the A/B knobs of r4c.sh.
source ./tools/gpu/step.sh
export TMPDIR=/tmp
step 600 r4d_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_user_operator.py tests/test_gpu_transpose.py tests/test_gpu_solver.py tests/test_gpu_chebyshev.py tests/test_gpu_formats.py
tail -3 gpurun_out/r4d_tests.log
for nz in 256 128 64 32; do
  VAR=MIGMRES_LD_PAD VALUES="64 128 256 320 512 576 1024 8256" ARGS="--nz $nz --no-csr-spmm" TAG=r4d_pad$nz bash tools/gpu/sweep.sh > /dev/null || exit 1
done
cat gpurun_out/sweep_r4d_pad*.txt
bash tools/gpu/r4c.sh
