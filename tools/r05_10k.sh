#!/bin/bash
# GPU box: dual suites (per-lane counters), then the 10,000-locus cfg5 batch
# with the wave kernels at 2 and at 1 wave per SIMD
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dual.py tests/test_priority_extras.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
W1=$PWD/waffle_con_amd/libwaffle_con_w1.so
for v in w2 w1; do
  if [ $v = w1 ]; then export WAFFLE_CON_LIB=$W1; fi
  timeout -k 10 400 python3 -u bench.py --workload cfg5 --loci 10000 --steps 1 --warmup 1 --no-cpu > $O/c5_$v.json 2> $O/c5_$v.err || { tail -5 $O/c5_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c5_$v.json'));print('$v', d['value'], d.get('loci_per_s'), d['ms_per_step'], d['kernel_ms_per_step'])"
done
