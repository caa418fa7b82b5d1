source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-nw16d}
step 120 mb_k16_${P}_m1.log ./tools/mb_k16 256
MIGMRES_NW16=3 step 120 mb_k16_${P}_m3.log ./tools/mb_k16 256
MIGMRES_NW16=3 MIGMRES_NW16_PF2=1 step 120 mb_k16_${P}_m3pf.log ./tools/mb_k16 256
MIGMRES_NW16=3 MIGMRES_NW16_PF2=1 step 600 pytest_nw16_${P}_m3pf.log python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_loopback.py -m gpu -x -q --timeout 300 --timeout-method thread -k "k16 or 16"
step 300 bench_${P}.json python bench.py --no-cpu-baseline
