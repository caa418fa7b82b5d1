source ./tools_gpu_check.sh
step 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
B="python bench.py --no-cpu-baseline"
for i in 1 2; do
  step 300 ab_old_$i.json env MIGMRES_SPEC_SPMM=0 $B
  step 300 ab_new_$i.json $B
done
step 300 ab_s128old.json env MIGMRES_SPEC_SPMM=0 $B --nx 128 --steps 200 --warmup 50
step 300 ab_s128new.json $B --nx 128 --steps 200 --warmup 50
