source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3m}
MIGMRES_NT_PW=2 step 200 mbk16_pw_$P.log ./tools/mb_k16
MIGMRES_NT_PW=0 step 200 mbk16_old_$P.log ./tools/mb_k16
step 120 pmc_k16_$P.log timeout -s KILL 110 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS -T --output-format csv -d gpurun_out/pmc_k16_$P -o run --kernel-include-regex "nn_tn" -- ./tools/mb_k16
step 300 bench_k16_$P.json python bench.py --no-cpu-baseline --k 16
