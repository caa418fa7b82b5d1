# GPU suite, ICGS vs DGKS headline (same box), Brick3D+Jacobi rocprof stats + SpMM PMC passes
source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3b}
rm -f gpurun_out/parity_margins.jsonl
step 600 pytest_gpu_$P.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
cp gpurun_out/parity_margins.jsonl gpurun_out/parity_margins_$P.jsonl
step 300 bench_icgs_$P.json python bench.py --no-cpu-baseline
step 300 bench_dgks_$P.json python bench.py --no-cpu-baseline --ortho DGKS
step 300 bench_bj_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
BJ="python3 bench.py --no-cpu-baseline --no-profile --matrix Brick3D --prec right --steps 25 --warmup 25"
step 300 rocprof_bj_$P.log rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_bj_$P -o run -- $BJ
step 120 pmc_bj_fetch_$P.log timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/pmc_bj_fetch_$P -o run --kernel-include-regex "spmm" -- $BJ
step 120 pmc_bj_write_$P.log timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d gpurun_out/pmc_bj_write_$P -o run --kernel-include-regex "spmm" -- $BJ
step 120 pmc_bj_tcc_$P.log timeout -s KILL 110 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum -T --output-format csv -d gpurun_out/pmc_bj_tcc_$P -o run --kernel-include-regex "spmm" -- $BJ
step 120 pmc_bj_sq_$P.log timeout -s KILL 110 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES -T --output-format csv -d gpurun_out/pmc_bj_sq_$P -o run --kernel-include-regex "spmm" -- $BJ
step 120 pmc_bj_ta_$P.log timeout -s KILL 110 rocprofv3 --pmc TA_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE -T --output-format csv -d gpurun_out/pmc_bj_ta_$P -o run --kernel-include-regex "spmm" -- $BJ
