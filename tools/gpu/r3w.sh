source ./tools/gpu/step.sh
P=${PROF:-r3w}
for b in m15_gs0 m15_gs1 m4_gs1 m12_gs1; do
  step 120 mbnntn_${b}_$P.log ./tools/mb_nntn_$b
  sed "s/^/$b /" gpurun_out/mbnntn_${b}_$P.log >> gpurun_out/mbnntn_all_$P.log
done
cat gpurun_out/mbnntn_all_$P.log
