set -o pipefail
O=gpurun_out/r02aa
mkdir -p $O
for v in main split; do
  if [ $v = main ]; then unset WAFFLE_CON_LIB; else export WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_$v.so; fi
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-e2e > $O/cfg2_$v.json 2> $O/cfg2_$v.err || { echo "cfg2 $v failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg2_$v.json')); print('$v cfg2 loci/s', d['loci_per_s'], 'kernel ms', d['kernel_ms_per_step'])"
  timeout -k 10 200 python -u bench.py --workload cfg3 --loci 768 --steps 1 --warmup 1 --no-cpu --no-e2e > $O/cfg3_$v.json 2> $O/cfg3_$v.err || { echo "cfg3 $v failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg3_$v.json')); print('$v cfg3 loci/s', d['loci_per_s'], 'kernel ms', d['kernel_ms_per_step'])"
done
