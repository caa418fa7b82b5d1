source ./tools_gpu_check.sh
for nb in 8 4 12 16 8; do step 120 mb_lib_nb$nb.log ./tools/mb_lib_nb$nb 256 64; done
