#!/bin/bash
# GPU box, final state: whole GPU suite + smoke, the cfg2 profile passes
# (kernel trace, HBM traffic, issue view), the cfg5 kernel trace, the default bench line
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
PASSES="kt fetch write sq1" bash tools/profile_round.sh ${T} --cfg5-loci 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -2 $O/prof.log
mkdir -p gpurun_out/prof_${T}c5
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}c5/kt -o run -- \
  python3 bench.py --workload cfg5 --loci 10000 --steps 1 --warmup 1 --no-cpu > gpurun_out/prof_${T}c5/kt_bench.json 2> $O/c5prof.err || { tail -5 $O/c5prof.err; exit 1; }
echo "cfg5 kt done"
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/bench.json'))
c=d['cfg5_strong']
print('value', d['value'], 'loci/s', d['loci_per_s'], 'ms', d['ms_per_step'], 'e2e', d.get('e2e_loci_per_s'))
print('cfg5', c['cfg5_loci_per_s'], c['elapsed_s'], c['tail']['projected_8gpu_eff'])"
