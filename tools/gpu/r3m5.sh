# uniform 27-point march (k_spmm_march27): parity, SpMM timing vs the lane-shared template kernel, Brick3D + Jacobi bench
source ./tools/gpu/step.sh
P=${PROF:-r3m5}
step 600 tests_$P.log python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_prec.py tests/test_gpu_loopback.py tests/test_gpu_formats.py -k "march or fused or distributed_spmm or spmm_bit or formats"
MIGMRES_NO_MARCH=1 step 120 ts_bk_tpl3_$P.log python tools/time_spmm.py Brick3D 256 8
for pd in 1 2 3; do
  MIGMRES_MARCH_PD=$pd step 120 ts_bk_pd${pd}_$P.log python tools/time_spmm.py Brick3D 256 8
done
MIGMRES_MARCH27_TABLE=1 step 120 ts_bk_table_$P.log python tools/time_spmm.py Brick3D 256 8
step 120 ts_bk384_$P.log python tools/time_spmm.py Brick3D 384 8
MIGMRES_NO_MARCH=1 step 120 ts_bk384_tpl3_$P.log python tools/time_spmm.py Brick3D 384 8
step 300 bench_bj_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
MIGMRES_NO_MARCH=1 step 300 bench_bj_nomarch_$P.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
for f in gpurun_out/ts_*_$P.log; do echo "$(basename $f .log): $(grep Brick3D $f)"; done
for f in bj bj_nomarch; do tail -1 gpurun_out/bench_${f}_$P.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', round(d['value'],2), d['kernels'].get('spmm'))"; done
