source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-r2e}
step 300 rocprof_k16_$P.log rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_k16_$P -o run -- python3 bench.py --no-cpu-baseline --k 16 --steps 25 --warmup 25 --no-profile
step 300 rocprof_bj_$P.log rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_bj_$P -o run -- python3 bench.py --no-cpu-baseline --matrix Brick3D --prec right --steps 25 --warmup 25 --no-profile
step 200 bench_k16_$P.log python bench.py --no-cpu-baseline --k 16
step 200 bench_bj_$P.log python bench.py --no-cpu-baseline --matrix Brick3D --prec right
