#!/bin/bash
# GPU box: whole GPU suite, smoke, 5949 critical path, cfg5 10k batch
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python3 -u tools/critical_path.py --top 0 --seeds 5949 887 --out $O/cp > $O/cp.log 2>&1 || { tail -5 $O/cp.log; exit 1; }
grep wall_s $O/cp.log
timeout -k 10 400 python3 -u bench.py --workload cfg5 --loci 10000 --steps 1 --warmup 1 --no-cpu > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c5.json'));print('cfg5 10k', d['value'], d.get('loci_per_s'), d['ms_per_step'], d['kernel_ms_per_step'])"
