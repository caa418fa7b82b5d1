source ./tools_gpu_check.sh
export TMPDIR=/tmp
step 600 bench_r1.log python bench.py
step 900 rocprof_stats.log rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_r1c -o run -- python3 bench.py --no-cpu-baseline
step 900 rocprof_fetch.log rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/prof_r1c_fetch -o run --kernel-include-regex "gemm_tn|nn_tn|gemm_nn|spmm|k_fb" -- python3 bench.py --no-cpu-baseline --no-profile
step 900 rocprof_write.log rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d gpurun_out/prof_r1c_write -o run --kernel-include-regex "gemm_tn|nn_tn|gemm_nn|spmm|k_fb" -- python3 bench.py --no-cpu-baseline --no-profile
