#!/bin/bash
# -s expansion: item setup only (M_ABL_NOEXP variant) vs full
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in base noexp; do
  if [ $v = noexp ]; then export A5X_LIB_PATH=$GRAFT_REPO_ROOT/hashcat_a5_table_generator_amd/_build_mnoexp/liba5x.so; fi
  timeout -k 10 300 python bench.py --mode 2 --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bo_$v.json 2> gpurun_out/bo_$v.err || { tail -3 gpurun_out/bo_$v.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/bo_$v.json'));r=d['roofline'];print('$v expand %.1f ms ks %.1f ms'%(r['ms_per_launch'],r['ms_keyspace_scan_plan']))"
done
