#!/bin/bash
# GPU box: whole GPU suite + smoke, then the cfg4 bench line
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 -u bench.py --workload cfg4 --steps 2 --warmup 1 --no-cpu > $O/cfg4.json 2> $O/cfg4.err || { tail -20 $O/cfg4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg4.json'));print('cfg4', d['ms_per_step'])"
