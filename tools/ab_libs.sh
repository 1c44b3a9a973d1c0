#!/bin/bash
# GPU box: A/B of library variants (waffle_con_amd/libwaffle_con_<v>.so) on
# one bench workload, alternating, on one box
#   bash tools/ab_libs.sh <tag> <workload> <reps> <v1> <v2> ...
export TMPDIR=/tmp
O=gpurun_out/$1
W=$2
N=$3
shift 3
mkdir -p $O
for rep in $(seq $N); do
  for v in "$@"; do
    WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_$v.so timeout -k 10 300 python3 -u bench.py --workload $W --steps 3 --warmup 1 --no-cpu --no-e2e $AB_ARGS > $O/${W}_${v}_$rep.json 2> $O/${W}_${v}_$rep.err || { tail -20 $O/${W}_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${W}_${v}_$rep.json'));print('$v', $rep, round(d['value']/1e6,1), d.get('loci_per_s'), round(d['ms_per_step'],1))"
  done
done
