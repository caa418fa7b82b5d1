# PMC of the plane-march SpMM kernels (what bounds k_spmm_march7 / k_spmm_march27): SQ instruction
# mix and waits, texture / L2 counters; one counter group per rocprofv3 pass
source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3f6}
for kind in Laplace3D Brick3D; do
  step 90 pmc_sq_${kind}_$P.log timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU -T --output-format csv -d gpurun_out/pmc_sq_${kind}_$P -o run --kernel-include-regex "march" -- python3 tools/time_spmm.py $kind 256 8 x 10
  step 90 pmc_tx_${kind}_$P.log timeout -s KILL 80 rocprofv3 --pmc TA_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum -T --output-format csv -d gpurun_out/pmc_tx_${kind}_$P -o run --kernel-include-regex "march" -- python3 tools/time_spmm.py $kind 256 8 x 10
  step 90 pmc_lds_${kind}_$P.log timeout -s KILL 80 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD -T --output-format csv -d gpurun_out/pmc_lds_${kind}_$P -o run --kernel-include-regex "march" -- python3 tools/time_spmm.py $kind 256 8 x 10
done
ls gpurun_out/pmc_*_$P
