#!/bin/bash
# GPU box: wave-engine phase profile of the 5949 full-read level, per-locus
# latency of the 2000-locus cfg5 batch (wave engine), cfg3 A/B, e2e bench line
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
WC_WAVE=1 WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg5-full --seed 5949 --phases /tmp/ph_1.txt > $O/full_1.log 2>&1 || { tail -20 $O/full_1.log; exit 1; }
grep -v amdgpu.ids $O/full_1.log
WC_WAVE=1 timeout -k 10 300 python3 -u tools/cfg5_lat.py --loci 2000 --out $O/lat1 > $O/lat1.log 2>&1 || { tail -20 $O/lat1.log; exit 1; }
grep -v amdgpu.ids $O/lat1.log
for eng in 0 1; do
  WC_WAVE=$eng timeout -k 10 300 python3 -u bench.py --workload cfg3 --steps 3 --warmup 1 --no-cpu > $O/c3_$eng.json 2> $O/c3_$eng.err || exit 1
  python3 -c "import json;d=json.load(open('$O/c3_$eng.json'));print('cfg3', $eng, d['value'], d.get('loci_per_s'), d['ms_per_step'], d['kernel_ms_per_step'])"
done
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d.get('e2e_loci_per_s'), d.get('e2e_upload_ms'), d.get('e2e_compute_ms'), d.get('e2e_upload_packed_bytes'))"
