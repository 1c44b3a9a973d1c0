#!/bin/bash
# GPU box: the engine-build and packed-upload parity tests, then the default
# bench line with the packed upload (default) and with WC_PACK=0
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_upload.py tests/test_gpu_builds.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for p in d 0; do
  if [ $p = 0 ]; then export WC_PACK=0; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu > $O/bench_$p.json 2> $O/bench_$p.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_$p.json'));print('$p', d['value'], d.get('e2e_loci_per_s'), d.get('e2e_upload_ms'), d.get('e2e_compute_ms'), d.get('e2e_upload_packed_bytes'))"
done
