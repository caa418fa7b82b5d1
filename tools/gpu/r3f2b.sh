# round-3 final state: rocprofv3 kernel stats + FETCH/WRITE PMC passes of the default bench, secondary benches
source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3f2}
step 600 rocprof_stats_$P.log rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_$P -o run -- python3 bench.py --no-cpu-baseline
find gpurun_out/prof_$P -type f ! -name '*stats*' -delete
step 300 rocprof_fetch_$P.log timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/prof_${P}_fetch -o run --kernel-include-regex "gemm_tn|nn_tn|gemm_nn|spmm|k_fb" -- python3 bench.py --no-cpu-baseline --no-profile
step 300 rocprof_write_$P.log timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d gpurun_out/prof_${P}_write -o run --kernel-include-regex "gemm_tn|nn_tn|gemm_nn|spmm|k_fb" -- python3 bench.py --no-cpu-baseline --no-profile
step 300 bench_k16_$P.json python bench.py --no-cpu-baseline --k 16
step 300 bench_bj_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
step 300 bench_flan_$P.json python bench.py --no-cpu-baseline --matrix FlanProxy --k 4
step 300 bench_dgks_$P.json python bench.py --no-cpu-baseline --ortho DGKS
step 300 bench_128_$P.json python bench.py --no-cpu-baseline --nx 128
step 300 bench_cheb_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right --prec-type chebyshev
for f in k16 bj flan dgks 128 cheb; do tail -1 gpurun_out/bench_${f}_$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value'],2), d['roofline']['kernel'], round(d['roofline']['frac'],3))"; done
