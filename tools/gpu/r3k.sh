source ./tools/gpu/step.sh
export TMPDIR=/tmp
P=${PROF:-r3k}
MIGMRES_NT_PW=1 step 200 mbk16_pw_$P.log ./tools/mb_k16
