source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3final}
step 600 rocprof_stats_$P.log rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_$P -o run -- python3 bench.py --no-cpu-baseline
find gpurun_out/prof_$P -type f ! -name '*stats*' -delete
step 300 rocprof_fetch_$P.log timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/prof_${P}_fetch -o run --kernel-include-regex "gemm_tn|nn_tn|gemm_nn|spmm|k_fb" -- python3 bench.py --no-cpu-baseline --no-profile
step 300 rocprof_write_$P.log timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d gpurun_out/prof_${P}_write -o run --kernel-include-regex "gemm_tn|nn_tn|gemm_nn|spmm|k_fb" -- python3 bench.py --no-cpu-baseline --no-profile
