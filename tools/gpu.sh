#!/bin/bash
# One runner for every GPU-box job (run through gpurun from the repo root):
#   bash tools/gpu.sh tests  <tag> [pytest args]      pytest -m gpu (default: whole suite)
#   bash tools/gpu.sh check  <tag> <lib> [pytest args] a bounds-checked library variant (make check)
#   bash tools/gpu.sh bench  <tag> [bench.py args]    one bench line -> gpurun_out/<tag>/bench.json
#   bash tools/gpu.sh profile <tag> [bench.py args]   tools/profile_round.sh (kernel trace + PMC passes)
#   bash tools/gpu.sh smoke  <tag>                    __graft_entry__.smoke()
#   bash tools/gpu.sh cmd    <tag> <seconds> <cmd...> any command under its own time limit
#   bash tools/gpu.sh ab     <tag> <workload> <reps> <v1> <v2> ...
#                                  library variants (waffle_con_amd/libwaffle_con_<v>.so,
#                                  "main" = libwaffle_con.so) alternating on one box, one
#                                  bench line each; AB_ARGS adds bench.py arguments
#   bash tools/gpu.sh sub    <tag> <variant> [one_sub.py args]   one sub-problem alone
#                                  (tools/one_sub.py) on a library variant
#   bash tools/gpu.sh pmc    <tag> <seconds> "<counters>" <cmd...>  one rocprofv3 --pmc pass
# Environment variables given to gpu.sh (WAFFLE_CON_LIB, WC_*) apply to every job;
# `cmd <tag> <s> env K=V prog` sets them for one job.
# Jobs can be chained: bash tools/gpu.sh tests t1 -- bench t1 --workload cfg5
# Every GPU step has its own timeout; the first failing step ends the call.
set -o pipefail
export TMPDIR=/tmp
run_job() {
  local job=$1 tag=$2
  shift 2
  local O=gpurun_out/$tag
  mkdir -p $O
  case $job in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread "$@" \
        > $O/pytest_gpu.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest_gpu.log; return 1; }
      tail -2 $O/pytest_gpu.log ;;
    check)
      local lib=$1
      shift
      WAFFLE_CON_LIB=$PWD/$lib timeout -k 10 900 python -u -m pytest -s -x -v --timeout 300 --timeout-method thread "$@" \
        > $O/check.log 2>&1 || { echo "check run failed"; grep -a "wc-check\|FAIL\|Error\|error" $O/check.log | head -40; tail -20 $O/check.log; return 1; }
      grep -a "wc-check" $O/check.log | head -20 || true
      tail -3 $O/check.log ;;
    bench)
      timeout -k 10 900 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err \
        || { echo "bench failed"; tail -30 $O/bench.err; return 1; }
      tail -c 3000 $O/bench.json ;;
    profile)
      bash tools/profile_round.sh $tag "$@" > $O/profile.log 2>&1 || { echo "profile failed"; tail -30 $O/profile.log; return 1; }
      tail -3 $O/profile.log ;;
    cmd)  # cmd <tag> <seconds> <command...>: any program, its own time limit, output in cmd.log
      local lim=$1
      shift
      timeout -k 10 $lim "$@" > $O/cmd.log 2>&1 || { echo "cmd failed: $*"; tail -30 $O/cmd.log; return 1; }
      tail -5 $O/cmd.log ;;
    ab)
      local W=$1 N=$2
      shift 2
      for rep in $(seq $N); do
        for v in "$@"; do
          local lib=$PWD/waffle_con_amd/libwaffle_con_$v.so
          [ "$v" = main ] && lib=$PWD/waffle_con_amd/libwaffle_con.so
          WAFFLE_CON_LIB=$lib timeout -k 10 400 python3 -u bench.py --workload $W --steps 3 --warmup 1 --no-cpu --no-e2e \
            $AB_ARGS > $O/${W}_${v}_$rep.json 2> $O/${W}_${v}_$rep.err || { echo "ab $v failed"; tail -20 $O/${W}_${v}_$rep.err; return 1; }
          python3 -c "import json;d=json.load(open('$O/${W}_${v}_$rep.json'));print('$v', $rep, round(d['value']/1e6,1), d.get('loci_per_s'), round(d['ms_per_step'],2), round(d['kernel_ms_per_step'],2))"
        done
      done ;;
    sub)
      local v=$1
      shift
      local lib=$PWD/waffle_con_amd/libwaffle_con_$v.so
      [ "$v" = main ] && lib=$PWD/waffle_con_amd/libwaffle_con.so
      WAFFLE_CON_LIB=$lib timeout -k 10 300 python3 -u tools/one_sub.py "$@" > $O/sub_$v.log 2>&1 \
        || { echo "sub failed"; tail -20 $O/sub_$v.log; return 1; }
      grep -v amdgpu $O/sub_$v.log | tail -3 ;;
    pmc)
      local lim=$1 ctrs=$2
      shift 2
      timeout -s KILL $lim rocprofv3 --pmc $ctrs --output-format csv -d $O/pmc -o run -- "$@" > $O/pmc.log 2>&1 \
        || { echo "pmc pass failed"; tail -20 $O/pmc.log; return 1; }
      echo "pmc done" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
        || { echo "smoke failed"; tail -30 $O/smoke.log; return 1; }
      tail -2 $O/smoke.log ;;
    *) echo "unknown job $job"; return 2 ;;
  esac
}
# split the arguments on "--" into jobs
args=()
for a in "$@"; do
  if [ "$a" = "--" ]; then
    run_job "${args[@]}" || exit 1
    args=()
  else
    args+=("$a")
  fi
done
[ ${#args[@]} -gt 0 ] && { run_job "${args[@]}" || exit 1; }
exit 0
