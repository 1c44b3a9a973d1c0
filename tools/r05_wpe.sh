#!/bin/bash
# GPU box: the two-reads-per-lane wave kernel at 1 (w1) vs 2 (w2) waves per
# SIMD: the 10,000-locus cfg5 batch and one 80-read sub-problem alone
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for v in w1 w2; do
  WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_$v.so timeout -k 10 300 python3 -u bench.py --workload cfg5 --loci 10000 --steps 1 --warmup 1 --no-cpu > $O/c5_$v.json 2> $O/c5_$v.err || { tail -20 $O/c5_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c5_$v.json'));print('$v', d['value'], d['ms_per_step'])"
  WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_$v.so timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg5-full --seed 1525 > $O/s1525_$v.log 2>&1 || exit 1
  echo $v $(grep us_per_pop $O/s1525_$v.log | python3 -c "import sys,json;d=json.loads(sys.stdin.read());print(d['us_per_pop'])")
done
