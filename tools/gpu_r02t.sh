#!/bin/bash
# stamps: with and without global stores (does the window setup wait drain the stores?)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
P=hashcat_a5_table_generator_amd
for v in diag diag4 diag; do
  A5X_LIB_PATH=$P/_build_$v/liba5x.so timeout -k 10 120 python tools/stamps.py c3 2000000 > gpurun_out/stamps_$v.txt 2>&1 || { tail -5 gpurun_out/stamps_$v.txt; exit 12; }
  echo "== $v"; cat gpurun_out/stamps_$v.txt
done
