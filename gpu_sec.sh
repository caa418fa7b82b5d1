source ./tools_gpu_check.sh
B="python bench.py --no-cpu-baseline"
step 300 sec_k16.json $B --k 16 --steps 50 --warmup 26
step 300 sec_brick.json $B --matrix Brick3D --steps 50 --warmup 25
step 300 sec_pseudo.json $B --solver GMRES --steps 50 --warmup 10
step 300 sec_flexjac.json $B --solver "FLEXIBLE GMRES" --prec right --steps 50 --warmup 25
step 300 sec_dgks.json $B --ortho DGKS --steps 50 --warmup 25
step 300 sec_main.json $B
