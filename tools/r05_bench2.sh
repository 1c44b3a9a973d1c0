#!/bin/bash
# GPU box: the default bench line
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/bench.json'))
c=d['cfg5_strong']
print('value', d['value'], 'loci/s', d['loci_per_s'], 'ms', d['ms_per_step'], 'kernel', d['roofline']['kernel_ms_per_launch'], 'e2e', d.get('e2e_loci_per_s'))
print('cfg5', c['cfg5_loci_per_s'], c['elapsed_s'], json.dumps(c['tail']))"
