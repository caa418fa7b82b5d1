source ./tools_gpu_check.sh
for v in a c; do step 60 mb_nntn_pf$v.log ./tools/mb_nntn_pf$v; done
step 120 mb_lib.log ./tools/mb_lib 256 64
