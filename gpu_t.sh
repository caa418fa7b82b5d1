source ./tools_gpu_check.sh
step 300 b128.json python bench.py --nx 128 --no-cpu-baseline --steps 200 --warmup 50
step 300 b161.json python bench.py --nx 161 --no-cpu-baseline --steps 200 --warmup 50
