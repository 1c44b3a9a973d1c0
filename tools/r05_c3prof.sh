#!/bin/bash
# GPU box: kernel-trace summary of the cfg3 bench (dual engine, 8-lane groups)
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- python3 -u bench.py --workload cfg3 --steps 3 --warmup 1 --no-cpu --no-e2e > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));print(d['value'],d.get('loci_per_s'),d['ms_per_step'])"
