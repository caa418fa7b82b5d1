source ./tools_gpu_check.sh
B="python bench.py --no-cpu-baseline"
for i in 1 2; do
  step 300 ab_old_$i.json bash -c "cd ab_old && $B"
  step 300 ab_new_$i.json $B
done
