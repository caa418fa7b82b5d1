# Round-4 session h: full GPU suite; 7-point march tile height (NL) A/B with FETCH/WRITE PMC
source ./tools/gpu/step.sh
export TMPDIR=/tmp
rm -f gpurun_out/parity_margins.jsonl
step 900 pytest_gpu_r4h.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
cp gpurun_out/parity_margins.jsonl gpurun_out/parity_margins_r4h.jsonl
tail -3 gpurun_out/pytest_gpu_r4h.log
VAR=MIGMRES_MARCH_NL VALUES="1 2 1 2" ARGS="--no-csr-spmm" TAG=r4h_nl bash tools/gpu/sweep.sh > /dev/null || exit 1
cat gpurun_out/sweep_r4h_nl.txt
for nl in 1 2; do
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmc_r4h_nl${nl}_$c
    MIGMRES_MARCH_NL=$nl step 120 pmc_r4h_nl${nl}_$c.log timeout -s KILL 100 rocprofv3 --pmc $c -T --output-format csv -d gpurun_out/pmc_r4h_nl${nl}_$c -o run --kernel-include-regex "spmm_march7" -- python3 bench.py --no-cpu-baseline --no-profile --no-csr-spmm --steps 25 --warmup 25
  done
done
python3 tools/pmc_kernels.py gpurun_out/pmc_r4h_nl1_ > gpurun_out/pmc_r4h_nl1.txt
python3 tools/pmc_kernels.py gpurun_out/pmc_r4h_nl2_ > gpurun_out/pmc_r4h_nl2.txt
cat gpurun_out/pmc_r4h_nl1.txt gpurun_out/pmc_r4h_nl2.txt
