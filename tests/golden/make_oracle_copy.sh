#!/bin/bash
# Build the scratch Python-3 copy of the reference used ONLY to generate the
# golden vectors (reference setup.py:98 installs with use_2to3=True; this does
# the same translation by hand).  Output goes to /tmp, never into the repo.
set -euo pipefail
DST=${DEAP_ORACLE_COPY:-/tmp/deap_oracle}
rm -rf "$DST"
mkdir -p "$DST/examples"
cp -r /root/reference/deap "$DST/"
cp -r /root/reference/examples/gp "$DST/examples/"
chmod -R u+w "$DST"
cd "$DST"
python3 -m lib2to3 -w -n deap examples/gp > /dev/null 2>&1
echo "reference copy ready at $DST"
