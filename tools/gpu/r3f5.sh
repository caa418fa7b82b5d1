# round-3 final tree: full GPU suite (parity margins logged), smoke, default bench with the CPU baseline
source ./tools/gpu/step.sh
P=${PROF:-r3f5}
rm -f gpurun_out/parity_margins.jsonl
step 1000 pytest_gpu_$P.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
cp gpurun_out/parity_margins.jsonl gpurun_out/parity_margins_$P.jsonl 2>/dev/null || true
step 300 smoke_$P.log python -c "import __graft_entry__ as g; g.smoke()"
step 400 bench_$P.log python bench.py
tail -2 gpurun_out/pytest_gpu_$P.log
