source ./tools/gpu/step.sh
P=${PROF:-r3x}
MIGMRES_NT_VIS32=1 step 300 mbk16_v32_$P.log ./tools/mb_k16x
MIGMRES_NT_VIS32=0 step 300 mbk16_v16_$P.log ./tools/mb_k16x
grep "k=16" gpurun_out/mbk16_v32_$P.log | sed 's/^/v32 /'
grep "k=16" gpurun_out/mbk16_v16_$P.log | sed 's/^/v16 /'
