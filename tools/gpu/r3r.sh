source ./tools/gpu/step.sh
P=${PROF:-r3r}
rm -f gpurun_out/parity_margins.jsonl
step 1000 tests_gpu_full_$P.log python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests
cp gpurun_out/parity_margins.jsonl gpurun_out/parity_margins_$P.jsonl 2>/dev/null || true
