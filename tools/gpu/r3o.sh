source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3o}
step 100 pmc_k16sq_$P.log timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T --output-format csv -d gpurun_out/pmc_k16sq_$P -o run --kernel-include-regex "nn_tn|gemm_tn" -- ./tools/mb_k16
