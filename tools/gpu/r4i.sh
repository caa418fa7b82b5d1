# Round-4 session i: full GPU suite, k = 16 timeline, secondary bench lines
source ./tools/gpu/step.sh
export TMPDIR=/tmp
rm -f gpurun_out/parity_margins.jsonl
step 900 pytest_gpu_r4i.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
cp gpurun_out/parity_margins.jsonl gpurun_out/parity_margins_r4i.jsonl
tail -3 gpurun_out/pytest_gpu_r4i.log
TAG=r4i_k16 ARGS="--k 16 --no-csr-spmm" ITERS=50 bash tools/gpu/trace.sh > /dev/null || exit 1
head -30 gpurun_out/timeline_r4i_k16.txt
step 300 bench_bj_r4i.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right
step 300 bench_flan_r4i.json python bench.py --no-cpu-baseline --matrix FlanProxy --k 4
step 300 bench_dgks_r4i.json python bench.py --no-cpu-baseline --ortho DGKS
step 300 bench_pseudo_r4i.json python bench.py --no-cpu-baseline --solver GMRES
step 300 bench_cheb_r4i.json python bench.py --no-cpu-baseline --matrix Brick3D --prec right --prec-type chebyshev
for f in bench_bj bench_flan bench_dgks bench_pseudo bench_cheb; do python3 tools/bench_summary.py gpurun_out/${f}_r4i.json $f; done
