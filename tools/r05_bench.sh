#!/bin/bash
# GPU box: the round's profile passes (cfg2 kernel trace + HBM traffic, cfg5
# kernel trace) and the default bench line
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T
mkdir -p $O
PASSES="kt fetch write sq1" bash tools/profile_round.sh ${T} --cfg5-loci 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -2 $O/prof.log
mkdir -p gpurun_out/prof_${T}c5
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}c5/kt -o run -- \
  python3 bench.py --workload cfg5 --loci 10000 --steps 1 --warmup 1 --no-cpu > gpurun_out/prof_${T}c5/kt_bench.json 2> $O/c5prof.err || { tail -5 $O/c5prof.err; exit 1; }
echo "cfg5 kt done"
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
for v in 2 1; do
  WC_WAVE=$v timeout -k 10 400 python3 -u bench.py --workload cfg4 --steps 1 --warmup 0 --no-cpu > $O/c4_$v.json 2> $O/c4_$v.err || { tail -5 $O/c4_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c4_$v.json'));print('cfg4 WC_WAVE=$v', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
done
