# wide dual engine register budget: 4 (128 VGPRs, spills), 3 (168), 2 (221, no spills) waves/SIMD
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_dw
mkdir -p $O
for v in dw2 dw3 base; do
  if [ $v = base ]; then L=$PWD/waffle_con_amd/libwaffle_con.so; else L=$PWD/waffle_con_amd/libwaffle_con_$v.so; fi
  WAFFLE_CON_LIB=$L timeout -k 10 300 python -u bench.py --workload cfg3 --steps 1 --warmup 1 --no-cpu > $O/cfg3_$v.json 2> $O/cfg3_$v.err || { echo "cfg3 $v failed"; tail $O/cfg3_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg3_$v.json')); print('$v cfg3 loci/s', round(d['loci_per_s'],1))"
  WAFFLE_CON_LIB=$L timeout -k 10 300 python -u bench.py --workload cfg4 --steps 1 --warmup 0 --no-cpu > $O/cfg4_$v.json 2> $O/cfg4_$v.err || { echo "cfg4 $v failed"; tail $O/cfg4_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg4_$v.json')); print('$v cfg4 s', round(d['ms_per_step']/1e3,2), 'kernel s', round(d['kernel_ms_per_step']/1e3,2))"
done
