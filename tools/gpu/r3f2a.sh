# round-3 final state (plane-march SpMM): march parity + SpMM timing, full GPU suite, smoke, default bench with CPU baseline
source ./tools/gpu/step.sh
P=${PROF:-r3f2}
step 300 tests_march_$P.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "march"
step 120 ts_uni7_$P.log python tools/time_spmm.py Laplace3D 256 8
MIGMRES_MARCH7_LANE_COEF=1 step 120 ts_lane7_$P.log python tools/time_spmm.py Laplace3D 256 8
step 120 ts_uni7_128_$P.log python tools/time_spmm.py Laplace3D 128 8
MIGMRES_MARCH_PD=2 step 120 ts_uni7pd2_$P.log python tools/time_spmm.py Laplace3D 256 8
rm -f gpurun_out/parity_margins.jsonl
step 1100 pytest_gpu_$P.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
cp gpurun_out/parity_margins.jsonl gpurun_out/parity_margins_$P.jsonl 2>/dev/null || true
step 300 smoke_$P.log python -c "import __graft_entry__ as g; g.smoke()"
step 400 bench_$P.log python bench.py
for f in gpurun_out/ts_*_$P.log; do echo "$(basename $f .log): $(grep Laplace3D $f)"; done
tail -2 gpurun_out/pytest_gpu_$P.log
