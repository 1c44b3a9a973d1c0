#!/bin/bash
# GPU box: whole GPU suite, smoke, the default bench line
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/bench.json'))
c=d['cfg5_strong']
print('value', d['value'], 'loci/s', d['loci_per_s'], 'e2e', d.get('e2e_loci_per_s'))
print('cfg5', c['cfg5_loci_per_s'], c['elapsed_s'], json.dumps(c['tail']))"
