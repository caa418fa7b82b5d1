source ./tools_gpu_check.sh
B="python bench.py --no-cpu-baseline"
step 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step 300 gram_new.json $B
step 300 gram_old.json env MIGMRES_FB_GRAM=0 $B
step 300 gram_new2.json $B
step 300 gram_old2.json env MIGMRES_FB_GRAM=0 $B
step 300 gram_s128new.json $B --nx 128 --steps 200 --warmup 50
step 300 gram_s128old.json env MIGMRES_FB_GRAM=0 $B --nx 128 --steps 200 --warmup 50
