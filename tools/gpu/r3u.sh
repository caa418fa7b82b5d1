source ./tools/gpu/step.sh
P=${PROF:-r3u}
for cfg in "0 8" "1 8" "1 4" "1 2" "0 4"; do
  set -- $cfg
  MIGMRES_TPL_SLABS=$1 MIGMRES_TPL_KC=$2 step 200 spmm7_s$1_kc$2_$P.log python tools/time_spmm.py Laplace3D 256 8
done
for cfg in "0 8" "1 8" "1 4"; do
  set -- $cfg
  MIGMRES_TPL_SLABS=$1 MIGMRES_TPL_KC=$2 step 200 spmm7k16_s$1_kc$2_$P.log python tools/time_spmm.py Laplace3D 256 16
done
grep -h "" gpurun_out/spmm7*_$P.log | grep -v amdgpu.ids
