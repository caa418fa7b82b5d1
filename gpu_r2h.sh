source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-r2h}
step 120 mb_k16_$P.log ./tools/mb_k16 256
step 1000 pytest_gpu_$P.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 300 smoke_$P.log python -c "import __graft_entry__ as g; g.smoke()"
step 400 bench_$P.log python bench.py
step 300 bench_k16_$P.json python bench.py --no-cpu-baseline --k 16
step 600 rocprof_k16_$P.log rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_k16_$P -o run -- python3 bench.py --no-cpu-baseline --k 16 --no-profile
step 300 rocprof_fetch_k16_$P.log timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/prof_k16_${P}_fetch -o run --kernel-include-regex "gemm_tn|nn_tn|gemm_nn|spmm|k_fb" -- python3 bench.py --no-cpu-baseline --no-profile --k 16
