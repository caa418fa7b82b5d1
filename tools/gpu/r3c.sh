# tpl3 (lane-shared 27-point SpMM) + fused Jacobi under halo: targeted tests, full suite, benches
source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3c}
rm -f gpurun_out/parity_margins.jsonl
step 300 pytest_tpl3_$P.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_loopback.py -x -v --timeout 120 --timeout-method thread -k "tpl3 or bit_exact or kernel_choice"
step 600 pytest_gpu_$P.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
cp gpurun_out/parity_margins.jsonl gpurun_out/parity_margins_$P.jsonl
step 300 bench_bj_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
step 300 bench_b_$P.json python bench.py --no-cpu-baseline --matrix Brick3D
MIGMRES_NO_TPL3=1 step 300 bench_bj_notpl3_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
BJ="python3 bench.py --no-cpu-baseline --no-profile --matrix Brick3D --prec right --steps 25 --warmup 25"
step 300 rocprof_bj_$P.log rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_bj_$P -o run -- $BJ
step 120 pmc_bj_ta_$P.log timeout -s KILL 110 rocprofv3 --pmc TA_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE -T --output-format csv -d gpurun_out/pmc_bj_ta_$P -o run --kernel-include-regex "spmm" -- $BJ
step 120 pmc_bj_sq_$P.log timeout -s KILL 110 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES -T --output-format csv -d gpurun_out/pmc_bj_sq_$P -o run --kernel-include-regex "spmm" -- $BJ
step 120 pmc_bj_fetch_$P.log timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/pmc_bj_fetch_$P -o run --kernel-include-regex "spmm" -- $BJ
