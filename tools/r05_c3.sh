#!/bin/bash
# GPU box: where a cfg3 locus's dual pops go on the block engine (one locus
# alone, normal and phase builds), then the cfg3 bench leg
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for seed in 0 1; do
  timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg3 --seed $seed > $O/s${seed}.log 2>&1 || exit 1
  grep us_per_pop $O/s${seed}.log
done
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg3 --seed 0 --phases /tmp/ph_c3.txt > $O/ph_c3.log 2>&1 || exit 1
grep -v amdgpu $O/ph_c3.log | tail -1
timeout -k 10 300 python3 -u bench.py --workload cfg3 --steps 3 --warmup 1 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));print(d['value'],d.get('loci_per_s'),d['ms_per_step'])"
