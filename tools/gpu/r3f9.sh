# march27 with the two-valued slot pattern fixed at compile time: parity, timing, Brick3D + Jacobi bench
source ./tools/gpu/step.sh
P=${PROF:-r3f9}
step 300 tests_$P.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_prec.py tests/test_gpu_loopback.py tests/test_gpu_formats.py -k "march or fused or spmm_bit or formats or tpl3"
step 120 ts_bk_$P.log python tools/time_spmm.py Brick3D 256 8
MIGMRES_MARCH27_TABLE=1 step 120 ts_bk_table_$P.log python tools/time_spmm.py Brick3D 256 8
step 300 bench_bj_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
for f in gpurun_out/ts_*_$P.log; do echo "$(basename $f .log): $(grep Brick3D $f)"; done
tail -1 gpurun_out/bench_bj_$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bj', round(d['value'],2), d['kernels'].get('spmm'))"
