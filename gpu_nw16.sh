source ./tools_gpu_check.sh
export TMPDIR=/tmp
P=${PROF:-nw16c}
for m in 1 3; do MIGMRES_NW16=$m step 120 mb_k16_${P}_m$m.log ./tools/mb_k16 256; done
MIGMRES_NW16=3 step 600 pytest_nw16_${P}_m3.log python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_loopback.py -m gpu -x -q --timeout 300 --timeout-method thread -k "k16 or 16"
for m in 1 3; do MIGMRES_NW16=$m step 300 bench_k16_${P}_m$m.json python bench.py --no-cpu-baseline --k 16; done
