source ./tools/gpu/step.sh
P=${PROF:-r3zb}
step 300 mbk16_pl_$P.log ./tools/mb_k16_pl
step 300 mbk16_nt_$P.log ./tools/mb_k16_nt
step 300 mbk16_pl2_$P.log ./tools/mb_k16_pl
paste <(grep "k= 8" gpurun_out/mbk16_pl_$P.log | awk '{print $2, $11, $13}') <(grep "k= 8" gpurun_out/mbk16_nt_$P.log | awk '{print $11, $13}') <(grep "k= 8" gpurun_out/mbk16_pl2_$P.log | awk '{print $11, $13}')
