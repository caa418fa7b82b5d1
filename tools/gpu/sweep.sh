# Same-box A/B sweep of one environment knob over bench.py lines.
#   VAR=MIGMRES_LD_PAD VALUES="64 512" ARGS="--nx 128" TAG=r4b bash tools/gpu/sweep.sh
# Writes gpurun_out/sweep_$TAG.txt: per value, it/s and the per-class GB/s.
source ./tools/gpu/step.sh
export TMPDIR=/tmp
T=${TAG:-sweep}
out=gpurun_out/sweep_$T.txt
: > $out
for v in $VALUES; do
  export $VAR=$v
  step 300 sweep_${T}_$v.json python bench.py --no-cpu-baseline --steps ${STEPS:-50} --warmup 25 $ARGS
  python tools/bench_summary.py gpurun_out/sweep_${T}_$v.json "$VAR=$v" >> $out
done
cat $out
