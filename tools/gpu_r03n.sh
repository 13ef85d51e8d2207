#!/bin/bash
# mode-engine layouts: parity (modes, long lines, C5 -s, CLI) + C5 -s bench
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_modes.py tests/test_gpu_long.py tests/test_gpu_cli.py tests/test_gpu_configs.py -q -m gpu -x --timeout 200 --timeout-method thread -k "mode or modes or cli or substitute or c5 or generate or long" > gpurun_out/tm.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tm.log
grep -E "Error|assert|FAILED" gpurun_out/tm.log | head -8
[ $rc -eq 0 ] || exit 10
for m in 2 3 1; do
timeout -k 10 300 python bench.py --mode $m --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bs_$m.json 2> gpurun_out/bs_$m.err || { tail -5 gpurun_out/bs_$m.err; exit 11; }
python -c "import json;d=json.load(open('gpurun_out/bs_$m.json'));r=d['roofline'];print('mode $m value %.3e cand/s step %.1f ms expand %.1f ms ks %.1f ms frac %.3f'%(d['value'],d['ms_per_step'],r['ms_per_launch'],r['ms_keyspace_scan_plan'],r['frac']))"
done
