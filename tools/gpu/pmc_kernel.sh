# PMC passes (one counter group per rocprofv3 run) for the kernels matching KRE in one bench
# command: FETCH/WRITE (HBM bytes), TA/TD busy, L2 hits/misses, SQ instruction mix.
#   TAG=r4c_flan KRE="spmm_bsr3|interleave" ARGS="--matrix FlanProxy --k 4" bash tools/gpu/pmc_kernel.sh
source ./tools/gpu/step.sh
export TMPDIR=/tmp
T=${TAG:-pmc}
K=${KRE:-spmm}
B="python3 bench.py --no-cpu-baseline --no-profile --no-csr-spmm --steps 25 --warmup 25 $ARGS"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_${T}_$i
  step 120 pmc_${T}_$i.log timeout -s KILL 100 rocprofv3 --pmc $grp -T --output-format csv -d gpurun_out/pmc_${T}_$i -o run --kernel-include-regex "$K" -- $B
done
python3 tools/pmc_kernels.py gpurun_out/pmc_${T}_ > gpurun_out/pmc_${T}.txt
cat gpurun_out/pmc_${T}.txt
