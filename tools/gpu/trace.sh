# Kernel-trace timeline of one bench configuration: bench line, rocprofv3 kernel trace,
# per-kernel / idle-gap summary (tools/timeline.py).  TAG names the outputs; ARGS are bench args.
#   TAG=r4a_128 ARGS="--nx 128" bash tools/gpu/trace.sh
source ./tools/gpu/step.sh
export TMPDIR=/tmp
T=${TAG:-trace}
A=${ARGS:-}
step 300 bench_$T.json python bench.py --no-cpu-baseline $A
rm -rf gpurun_out/tr_$T
step 300 trace_$T.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$T -o run -- python3 bench.py --no-cpu-baseline --no-profile $A
step 60 timeline_$T.txt python tools/timeline.py gpurun_out/tr_$T --iters ${ITERS:-100}
cat gpurun_out/timeline_$T.txt
