#!/bin/bash
# GPU box: the four-reads-per-lane wave kernel (WC_WAVE=2): dual suites and
# full-size cfg3 loci under it, then cfg3 with and without it
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
WC_WAVE=2 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dual.py tests/test_gpu_fullsize.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 2 1; do
  WC_WAVE=$v timeout -k 10 300 python3 -u bench.py --workload cfg3 --steps 3 --warmup 1 --no-cpu > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c3_$v.json'));print('cfg3 WC_WAVE=$v', d['value'], d.get('loci_per_s'), d['ms_per_step'], d['kernel_ms_per_step'])"
done
