#!/bin/bash
# GPU box: the engine-build and packed-upload parity tests, then the default
# bench line with the packed upload (default) and with WC_PACK=0
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_upload.py tests/test_gpu_builds.py tests/test_gpu_single.py -k 'upload or builds or cu' > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for p in d 0; do
  if [ $p = 0 ]; then export WC_PACK=0; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu > $O/bench_$p.json 2> $O/bench_$p.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$p.json'));print('$p', d['value'], d.get('e2e_loci_per_s'), d.get('e2e_upload_ms'), d.get('e2e_compute_ms'), d.get('e2e_upload_packed_bytes'))"
done
unset WC_PACK
if [ -n "$2" ]; then
  for eng in 1 0; do
    WC_WAVE=$eng WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg5-full --seed 5949 --phases /tmp/ph_$eng.txt > $O/full_$eng.log 2>&1 || exit 1
    cat $O/full_$eng.log
  done
  bash tools/r05_cfg5ab.sh $1_ab
fi
exit 0
