# launch paths with the plane-march SpMM: torchrun N=1, the one-rank RCCL transport at the 8-GPU
# per-rank size, pseudo-block GMRES; rocprofv3 kernel stats of Brick3D + Jacobi (k_spmm_march27)
source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3f3}
step 300 bench_torchrun1_$P.json python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 25 --warmup 25 --no-cpu-baseline
MIGMRES_FORCE_RCCL=1 step 300 bench_rccl128_$P.json python bench.py --no-cpu-baseline --nx 128
step 300 bench_pseudo_$P.json python bench.py --no-cpu-baseline --solver GMRES
step 600 rocprof_bj_$P.log rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_bj_$P -o run -- python3 bench.py --no-cpu-baseline --matrix Brick3D --prec right
find gpurun_out/prof_bj_$P -type f ! -name '*stats*' -delete
for f in torchrun1 rccl128 pseudo; do tail -1 gpurun_out/bench_${f}_$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value'],2), d['n_gpus'], d['config'].get('parallelism'), d['kernels'].get('spmm',{}).get('ms'))"; done
head -6 gpurun_out/prof_bj_$P/run_kernel_stats.csv
