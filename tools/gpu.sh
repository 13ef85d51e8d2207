#!/bin/bash
# tools/gpu.sh -- the one GPU-box script: runs the named steps in order, stops at the
# first failure (each GPU step under its own time limit).  Outputs go to gpurun_out/.
#
#   /usr/local/graft/bin/gpurun --timeout 900 -- 'TAG=r03a bash tools/gpu.sh test bench prof'
#
# steps (environment knobs in brackets):
#   test        pytest -m gpu [TESTS=paths, K=-k expr, TT=per-step seconds]
#   bench       one bench.py line -> gpurun_out/bench_$TAG$NAME.json [BENCH_ARGS, NAME]
#   ab          A/B of liba5x variants on one workload [VARIANTS="name:ENV=v,LIB=path ...",
#               STEPS, WORDS, WL, BENCH_ARGS]
#   prof        rocprofv3 --kernel-trace --stats of a short bench run [BENCH_ARGS]
#   traffic     PMC WRITE_SIZE / FETCH_SIZE of k_expand_fast -> gpurun_out/pmc_$TAG_$WL.json
#               [WL, WORDS, KRE]
#   pmc         PMC counter groups, one pass each (PMC="group\ngroup", KRE, BENCH_ARGS)
#   digestprof  fused-digest kernel stats + VALU counters [ALGOS, KRE, KNAME, WORDS, DARGS]
#               (modes: KRE="k_expand_fast_md5|k_mode_digest" KNAME="k_expand_fast_md5+k_mode_digest_*"
#               DARGS="--mode 3 --min 1")
#   stamps      per-phase cycle stamps (diagnostic build _build_diag) [WL, SW]
#   final       test + C3 bench (+ steady state, CPU baseline)/prof/traffic + C4 + C2a
#   final2      fused digests (+ dabl op breakdown) + C5 modes (+ rocprof) + stdout path
#   dabl        fused-digest VALU per candidate, product vs FX_DABL variant builds [ALGOS, WORDS]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
mkdir -p gpurun_out
T=${TAG:-x}

summ() {  # one-line summary of a bench JSON
  python3 - "$1" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d.get("roofline") or {}
extra = ""
if r.get("bound") == "hbm":
    extra = "expand %.2f ms %.0f GB/s frac %.3f ks %.2f ms" % (r["ms_per_launch"], r["achieved"], r["frac"],
                                                            r.get("ms_keyspace_scan_plan", 0))
elif r:
    extra = "%s frac %s" % (r.get("kernel"), r.get("frac"))
ss = d.get("steady_state")
if ss:
    extra += " | steady %.3e cand/s frac %.3f" % (ss["value"], ss["frac"])
c = d.get("cpu_baseline")
if "ms_per_step" not in d:  # the stdout line: one record per path
    print("%-28s value %.3e %s " % (sys.argv[1].split("/")[-1], d["value"], d["unit"]) + " ".join(
        "%s %.1f GB/s (pcie %.2f)" % (k, v["GB_per_s"], v["pcie_frac"]) for k, v in d.items()
        if isinstance(v, dict) and "GB_per_s" in v))
    sys.exit(0)
print("%-28s value %.3e %s step %.2f ms %s%s" % (sys.argv[1].split("/")[-1], d["value"], d["unit"], d["ms_per_step"],
                                              extra, (" cpu %.3e" % c["value"]) if c else ""))
PY
}

step_test() {
  timeout -k 10 ${TT:-600} python -u -m pytest ${TESTS:-tests/} -v -m gpu -x ${K:+-k "$K"} --timeout ${TTO:-200} \
    --timeout-method thread -rA --junitxml gpurun_out/junit_$T.xml > gpurun_out/test_$T.log 2>&1
  local rc=$?
  echo "pytest rc=$rc"; tail -2 gpurun_out/test_$T.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/test_$T.log | head -8; return 10; }
}

step_bench() {
  local f=gpurun_out/bench_$T${NAME}.json
  timeout -k 10 ${BT:-400} python bench.py ${BENCH_ARGS} > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; return 11; }
  summ $f
}

step_ab() {
  for v in ${VARIANTS:-"cur:X=0"}; do
    local name=${v%%:*} envs=${v#*:}
    ( IFS=','; for kv in $envs; do
        k=${kv%%=*}; val=${kv#*=}
        if [ "$k" = LIB ]; then export A5X_LIB_PATH=$R/$val; else export $k=$val; fi
      done
      unset IFS
      timeout -k 10 200 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --words ${WORDS:-10000000} \
        --workload ${WL:-c3} ${BENCH_ARGS} > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err ) \
      || { echo "bench $name failed"; tail -5 gpurun_out/ab_$name.err; return 12; }
    summ gpurun_out/ab_$name.json
  done
}

step_prof() {
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T \
      -o run --output-format csv -- python3 $R/bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline \
      ${BENCH_ARGS} > $R/gpurun_out/prof_$T.log 2>&1 ) || { tail -5 gpurun_out/prof_$T.log; return 13; }
  python3 - <<PY
import csv
for r in list(csv.DictReader(open("$R/gpurun_out/prof_$T/run_kernel_stats.csv")))[:8]:
    print("%-28s calls %4s avg %10.1f us total %8.2f ms %5s%%" % (r["Name"][:28], r["Calls"],
          float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6, r["Percentage"]))
PY
}

step_traffic() {  # [WL, WORDS, KRE, TMODE: -r / -s / -s -r (the expansion's k_expand_fast + item kernels summed)]
  local W=${WORDS:-10000000} WLx=${WL:-c3} M=${TMODE:-0}
  local ARGS="--steps 1 --warmup 0 --no-cpu-baseline --words $W --workload $WLx --mode $M --steady-batches 0"
  local K=${KRE:-k_expand_fast}
  [ "$M" != 0 ] && K=${KRE:-'k_expand_fast|k_mode_items_fast|k_mode_items_pos|k_mode_items_b\('}
  for grp in WRITE_SIZE FETCH_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$K" \
        -d $R/gpurun_out/pmct_${T}_$grp -o run --output-format csv -- python3 $R/bench.py $ARGS \
        > $R/gpurun_out/pmct_${T}_$grp.log 2>&1 ) || { echo "pmc $grp failed"; tail -5 gpurun_out/pmct_${T}_$grp.log; return 14; }
  done
  python3 tools/pmc_summary.py traffic "$T" "$WLx" "$W" "$K" "$M"
}

step_pmc() {
  local i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i + 1))
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "${KRE:-k_expand_fast}" \
        -d $R/gpurun_out/pmc_${T}_$i -o run --output-format csv -- python3 $R/bench.py \
        ${BENCH_ARGS:---steps 1 --warmup 0 --no-cpu-baseline --words 2000000} > $R/gpurun_out/pmc_${T}_$i.log 2>&1 ) \
      || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc_${T}_$i.log; return 15; }
  done <<GROUPS
${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH
GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL}
GROUPS
  python3 tools/pmc_summary.py mix gpurun_out/pmc_${T}_
}

step_digestprof() {
  local W=${WORDS:-2000000}
  for A in ${ALGOS:-md5 ntlm}; do
    local K=${KRE:-k_expand_fast_$A} KN=${KNAME:-${KRE:-k_expand_fast_$A}}
    local ARGS="--digest $A --workload c5 --words $W --no-cpu-baseline --targets 1000000 ${DARGS}"
    ( cd /tmp && export TMPDIR=/tmp &&
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/dprof_$A -o run --output-format csv -- \
        python3 $R/bench.py $ARGS --steps 2 --warmup 1 > $R/gpurun_out/dprof_$A.log 2>&1 &&
      timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex $K -d $R/gpurun_out/dpmc1_$A -o run --output-format csv -- \
        python3 $R/bench.py $ARGS --steps 1 --warmup 0 > $R/gpurun_out/dpmc1_$A.log 2>&1 ) \
      || { echo "digest prof $A failed"; tail -5 gpurun_out/dprof_$A.log gpurun_out/dpmc1_$A.log; return 16; }
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc VALUBusy VALUUtilization \
        --kernel-include-regex $K -d $R/gpurun_out/dpmc2_$A -o run --output-format csv -- \
        python3 $R/bench.py $ARGS --steps 1 --warmup 0 > $R/gpurun_out/dpmc2_$A.log 2>&1 ) \
      || echo "derived VALUBusy pass $A failed (raw counters only)"
    python3 tools/digest_prof_summary.py $A $W "$KN" || return 16
  done
}

step_dabl() {  # fused-digest op breakdown: VALU instructions per candidate with MD rounds / probe ablated
  local W=${WORDS:-2000000}
  for A in ${ALGOS:-md5 ntlm}; do
    for v in cur dabl1 dabl2 dabl3; do
      local lib=""
      [ $v != cur ] && lib=$R/hashcat_a5_table_generator_amd/_build_$v/liba5x.so
      ( cd /tmp && export TMPDIR=/tmp && A5X_BENCH_NO_HITCHECK=1 A5X_LIB_PATH=$lib timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES \
          --kernel-include-regex k_expand_fast_$A -d $R/gpurun_out/dabl_${A}_$v -o run --output-format csv -- \
          python3 $R/bench.py --digest $A --workload c5 --words $W --no-cpu-baseline --targets 1000000 --steps 1 --warmup 0 \
          > $R/gpurun_out/dabl_${A}_$v.log 2>&1 ) || { echo "dabl $A $v failed"; tail -5 gpurun_out/dabl_${A}_$v.log; return 18; }
    done
  done
  python3 tools/digest_prof_summary.py breakdown "${ALGOS:-md5 ntlm}"
}

step_ksab() {  # keyspace-only A/B of liba5x variants under rocprofv3 kernel stats [KSVARIANTS, WL, WORDS]
  for v in ${KSVARIANTS:-cur}; do
    local lib=""
    [ $v != cur ] && lib=$R/hashcat_a5_table_generator_amd/_build_$v/liba5x.so
    ( cd /tmp && export TMPDIR=/tmp && A5X_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats \
        -d $R/gpurun_out/ksab_${T}_$v -o run --output-format csv -- python3 $R/tools/ks_time.py ${WL:-c3} ${WORDS:-10000000} \
        > $R/gpurun_out/ksab_${T}_$v.log 2>&1 ) || { echo "ksab $v failed"; tail -3 gpurun_out/ksab_${T}_$v.log; return 19; }
    echo "-- $v: $(tail -1 gpurun_out/ksab_${T}_$v.log)"
    python3 - <<PY
import csv
for r in list(csv.DictReader(open("$R/gpurun_out/ksab_${T}_$v/run_kernel_stats.csv")))[:6]:
    print("   %-26s calls %3s avg %9.1f us" % (r["Name"][:26], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  done
}

step_stamps() {
  timeout -k 10 120 python tools/stamps.py ${WL:-c3} ${SW:-2000000} > gpurun_out/stamps_$T.txt 2>&1 \
    || { tail -5 gpurun_out/stamps_$T.txt; return 17; }
  cat gpurun_out/stamps_$T.txt
}

step_final() {  # part 1: tests, the headline C3 line and its evidence, C4, C2a, steady state
  TT=900 step_test || return $?
  NAME=_c3 BENCH_ARGS="" step_bench || return $?
  BENCH_ARGS="--steady-batches 0" step_prof || return $?
  WL=c3 step_traffic || return $?
  NAME=_c4 BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --workload c4 --words 12500000 --steady-batches 0" step_bench || return $?
  NAME=_c2a BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --workload c2a --words 1000000 --steady-batches 0" step_bench || return $?
}

step_final2() {  # part 2: fused digests (+ op breakdown), the -r / -s / -s -r lines and profiles, stdout path
  ALGOS="md5 ntlm" step_digestprof || return $?
  for alg in md5 ntlm; do
    NAME=_digest_$alg BENCH_ARGS="--digest $alg --workload c5 --words 2000000 --targets 1000000 --steps 3 --warmup 1" \
      step_bench || return $?
  done
  step_dabl || return $?
  for m in 1 2 3; do
    NAME=_c5_mode$m BENCH_ARGS="--mode $m --workload c5 --steps 3 --warmup 1 --no-cpu-baseline" step_bench || return $?
  done
  local T0=$T
  for m in 1 2; do
    T=${T0}_m$m; BENCH_ARGS="--mode $m --workload c5 --steady-batches 0" STEPS=2 step_prof || { T=$T0; return 13; }
  done
  T=$T0
  NAME=_stdout BENCH_ARGS="--stdout --no-cpu-baseline" step_bench || return $?
}

[ $# -gt 0 ] || set -- test
for s in "$@"; do
  echo "== step $s ($(date +%T))"
  "step_$s" || { rc=$?; echo "step $s failed (rc $rc)"; exit $rc; }
done
echo "== done ($(date +%T))"
