source ./tools/gpu/step.sh
P=${PROF:-r3t}
MIGMRES_SETUP_TRACE=1 step 300 fc_setup_$P.log python tools/time_fillcomplete.py Laplace3D 256 host_devfmt,device_devfmt
cat gpurun_out/fc_setup_$P.log
