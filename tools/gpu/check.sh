# GPU suite (margins logged) + smoke + headline bench.  PROF names the round/session.
source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3}
rm -f gpurun_out/parity_margins.jsonl
step 600 pytest_gpu_$P.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
cp gpurun_out/parity_margins.jsonl gpurun_out/parity_margins_$P.jsonl
step 120 smoke_$P.log python -c "import __graft_entry__ as g; g.smoke()"
step 400 bench_$P.json python bench.py
