# Round measurement session: full GPU suite (parity margins logged), smoke, the default bench
# line (CPU baseline included), the 8-GPU per-rank slice with the real one-rank RCCL
# communicator, rocprofv3 kernel stats of both, FETCH/WRITE PMC passes of the headline and the
# PMC summary bench.py reads.  PROF names the outputs.
source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r4f}
rm -f gpurun_out/parity_margins.jsonl
step 900 pytest_gpu_$P.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
cp gpurun_out/parity_margins.jsonl gpurun_out/parity_margins_$P.jsonl
tail -3 gpurun_out/pytest_gpu_$P.log
step 300 smoke_$P.log python -c "import __graft_entry__ as g; g.smoke()"
step 600 bench_$P.json python bench.py
MIGMRES_FORCE_RCCL=1 step 300 bench_rccl128_$P.json python bench.py --nx 128 --no-cpu-baseline
MIGMRES_FORCE_RCCL=1 step 300 rocprof_rccl128_$P.log rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_rccl128_$P -o run -- python3 bench.py --nx 128 --no-cpu-baseline --no-csr-spmm
step 300 rocprof_stats_$P.log rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_$P -o run -- python3 bench.py --no-cpu-baseline --no-csr-spmm
step 300 rocprof_fetch_$P.log timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/prof_${P}_fetch -o run --kernel-include-regex "gemm_tn|nn_tn|gemm_nn|spmm|k_fb" -- python3 bench.py --no-cpu-baseline --no-profile --no-csr-spmm
step 300 rocprof_write_$P.log timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d gpurun_out/prof_${P}_write -o run --kernel-include-regex "gemm_tn|nn_tn|gemm_nn|spmm|k_fb" -- python3 bench.py --no-cpu-baseline --no-profile --no-csr-spmm
python3 tools/timeline.py gpurun_out/prof_rccl128_$P > gpurun_out/timeline_rccl128_$P.txt
python3 tools/timeline.py gpurun_out/prof_$P > gpurun_out/timeline_$P.txt
grep -h '"value"' gpurun_out/bench_$P.json gpurun_out/bench_rccl128_$P.json | cut -c1-200
FE=$(ls gpurun_out/prof_${P}_fetch/*counter_collection.csv gpurun_out/prof_${P}_fetch/*/*counter_collection.csv 2>/dev/null | head -1)
WR=$(ls gpurun_out/prof_${P}_write/*counter_collection.csv gpurun_out/prof_${P}_write/*/*counter_collection.csv 2>/dev/null | head -1)
ST=$(ls gpurun_out/prof_$P/*kernel_stats.csv gpurun_out/prof_$P/*/*kernel_stats.csv 2>/dev/null | head -1)
python3 tools/pmc_summary.py "$FE" "$WR" "$ST" gpurun_out/pmc_summary_$P.json gpurun_out/bench_$P.json && python3 -c "
import json; d=json.load(open('gpurun_out/pmc_summary_$P.json'))
print({k: round(v.get('ratio') or 0, 4) for k, v in d['kernels'].items()})"
