source ./tools/gpu/step.sh
P=${PROF:-r3v}
for m in 15 13 14 12 4; do
  step 120 mbnntn_m${m}_$P.log ./tools/mb_nntn_m$m
done
cat gpurun_out/mbnntn_m*_$P.log
