source ./tools/gpu/step.sh
P=${PROF:-r3s}
for kind in "Laplace3D 256" "Brick3D 200" "FlanProxy 81"; do
  for v in host_hostfmt host_devfmt device_hostfmt device_devfmt; do
    step 300 fc_${v}_$P.json python tools/time_fillcomplete.py $kind $v
    tail -1 gpurun_out/fc_${v}_$P.json >> gpurun_out/fc_all_$P.jsonl
  done
done
cat gpurun_out/fc_all_$P.jsonl
