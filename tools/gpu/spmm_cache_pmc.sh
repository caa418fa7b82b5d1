source ./tools/gpu/step.sh
export TMPDIR=/tmp
step 120 pmc_a.log timeout -s KILL 100 rocprofv3 --pmc TA_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE -T --output-format csv -d gpurun_out/pmc_a -o run --kernel-include-regex "spmm|gemm_tn" -- python3 bench.py --no-cpu-baseline --no-profile --steps 25 --warmup 25
step 120 pmc_b.log timeout -s KILL 100 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum -T --output-format csv -d gpurun_out/pmc_b -o run --kernel-include-regex "spmm|gemm_tn" -- python3 bench.py --no-cpu-baseline --no-profile --steps 25 --warmup 25
