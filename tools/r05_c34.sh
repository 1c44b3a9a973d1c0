#!/bin/bash
# GPU box: the cfg3 and cfg4 bench lines on the final tree (with their CPU baselines)
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python3 -u bench.py --workload cfg3 --steps 3 --warmup 1 > $O/cfg3.json 2> $O/cfg3.err || { tail -20 $O/cfg3.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg3.json'));print('cfg3', d.get('loci_per_s'), d['ms_per_step'], d['cpu_baseline'].get('loci_per_s'))"
timeout -k 10 600 python3 -u bench.py --workload cfg4 --steps 2 --warmup 1 > $O/cfg4.json 2> $O/cfg4.err || { tail -20 $O/cfg4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg4.json'));print('cfg4', d['ms_per_step'], json.dumps(d['cpu_baseline'])[:300])"
