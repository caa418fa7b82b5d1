# checkpoint with the 7-point march: full GPU suite, smoke, default bench (with CPU baseline)
source ./tools/gpu/step.sh
P=${PROF:-r3s1}
rm -f gpurun_out/parity_margins.jsonl
step 1000 pytest_gpu_$P.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
cp gpurun_out/parity_margins.jsonl gpurun_out/parity_margins_$P.jsonl 2>/dev/null || true
step 300 smoke_$P.log python -c "import __graft_entry__ as g; g.smoke()"
step 400 bench_$P.log python bench.py
tail -3 gpurun_out/pytest_gpu_$P.log
