#!/bin/bash
# Build the library of a git revision (default HEAD) under ab_old/ for same-box A/B bench runs:
#   bash tools/mk_ab_old.sh [rev]; then: (cd ab_old && python bench.py) next to python bench.py
set -e
rev=${1:-HEAD}
rm -rf ab_old && mkdir -p ab_old/trilinos_amd/csrc ab_old/include ab_old/profiles
cp -r bench.py oracle ab_old/ && cp profiles/pmc_summary.json ab_old/profiles/
for f in $(git ls-files trilinos_amd include); do mkdir -p ab_old/$(dirname $f); git show $rev:$f > ab_old/$f; done
make -C ab_old/trilinos_amd/csrc -j8 > /dev/null
ls -la ab_old/trilinos_amd/libmigmres.so
