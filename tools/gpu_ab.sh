#!/bin/bash
# GPU-box script: A/B of expansion variants on the same workload (expand ms per variant).
# VARIANTS: space-separated "name:ENV=val,ENV=val" (LIB=path selects another liba5x build).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
for v in ${VARIANTS:-"cur:X=0"}; do
  name=${v%%:*}; envs=${v#*:}
  ( IFS=','; for kv in $envs; do
      k=${kv%%=*}; val=${kv#*=}
      if [ "$k" = LIB ]; then export A5X_LIB_PATH=$R/$val; else export $k=$val; fi
    done
    timeout -k 10 120 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --words ${WORDS:-10000000} --workload ${WL:-c3} > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err ) || { echo "bench $name failed"; tail -5 gpurun_out/ab_$name.err; exit 11; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$name.json'));r=d['roofline'];print('%-10s expand %.2f ms  %.0f GB/s  ks %.2f ms  step %.2f ms'%('$name',r['ms_per_launch'],r['achieved'],r['ms_keyspace_scan_plan'],d['ms_per_step']))"
done
