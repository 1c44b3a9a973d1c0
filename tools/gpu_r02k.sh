set -o pipefail
O=gpurun_out/r02k
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 170 --timeout-method thread -k "not cfg4_full" > $O/tests.log 2>&1
echo "tests rc=$?"
tail -3 $O/tests.log
for v in main d5 d6; do
  if [ $v = main ]; then unset WAFFLE_CON_LIB; else export WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_$v.so; fi
  timeout -k 10 200 python -u bench.py --workload cfg3 --loci 768 --steps 1 --warmup 1 --no-cpu > $O/cfg3_$v.json 2> $O/cfg3_$v.err || { echo "cfg3 $v failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg3_$v.json')); print('$v cfg3 loci/s', d['loci_per_s'], 'kernel ms', d['kernel_ms_per_step'])"
  timeout -k 10 300 python -u tools/priority_bench.py --loci 1024 --cpu-loci 4 > $O/prio_$v.json 2> $O/prio_$v.err || { echo "prio $v failed"; exit 1; }
  echo "$v prio"; cat $O/prio_$v.json
done
unset WAFFLE_CON_LIB
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python -u tools/phase_run.py --workload cfg5-hpc --loci 1024 --out $O/ph_cfg5 > $O/ph_cfg5.log 2>&1; echo "ph cfg5 rc=$?"
WC_LAUNCH_LOG=1 timeout -k 10 600 python -u bench.py --workload cfg4 --steps 1 --warmup 0 --no-cpu > $O/bench_cfg4.json 2> $O/bench_cfg4.err; echo "cfg4 rc=$?"
cat $O/bench_cfg4.json
