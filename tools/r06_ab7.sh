#!/bin/bash
# round 6 A/B 7: fused digest early rejection (prefilter on digest words 0 / 3 before the last two
# MD steps) -- digest tests, then C5 MD5 / NTLM / -s -r -m 1 MD5 lines vs the previous commit (base)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} || exit 2
mkdir -p gpurun_out
L=hashcat_a5_table_generator_amd/_build
echo "== digest tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_digest.py tests/test_gpu_configs.py tests/test_gpu_vwords.py -x -q -m gpu \
  -k "digest or fused or lookup or hit" --timeout 200 --timeout-method thread > gpurun_out/r06i_tests.log 2>&1 || { tail -20 gpurun_out/r06i_tests.log; exit 3; }
tail -1 gpurun_out/r06i_tests.log
for args in "--digest md5" "--digest ntlm" "--digest md5 --mode 3 --min 1"; do
  n=$(echo $args | tr -d ' -' )
  for v in base cur base2 cur2; do
    lib=""; [ ${v%2} = base ] && lib=$PWD/${L}_base/liba5x.so
    A5X_LIB_PATH=$lib timeout -k 10 200 python bench.py $args --workload c5 --words 2000000 --targets 1000000 --steps 3 --warmup 1 \
      --no-cpu-baseline > gpurun_out/r06i_${n}_$v.json 2> gpurun_out/r06i_${n}_$v.err || { tail -5 gpurun_out/r06i_${n}_$v.err; exit 4; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-28s %-6s value %.4e ms/step %.2f' % (sys.argv[2], sys.argv[3], d['value'], d['ms_per_step']))" gpurun_out/r06i_${n}_$v.json "$args" $v
  done
done
