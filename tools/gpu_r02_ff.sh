# quiet-step fast-forward in the chain walk + gstate dual back at 4 waves/SIMD
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_ff
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_builds.py -x -q --timeout 120 --timeout-method thread > $O/pytest_builds.log 2>&1 || { echo "build tests failed"; tail -30 $O/pytest_builds.log; exit 1; }
tail -1 $O/pytest_builds.log
true
true
for v in ff noff; do
  if [ $v = ff ]; then L=$PWD/waffle_con_amd/libwaffle_con.so; else L=$PWD/waffle_con_amd/libwaffle_con_noff.so; fi
  WAFFLE_CON_LIB=$L timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-e2e > $O/cfg2_$v.json 2> $O/cfg2_$v.err || { echo "cfg2 $v failed"; tail $O/cfg2_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg2_$v.json')); print('$v cfg2 loci/s', round(d['loci_per_s']), 'kernel ms', round(d['kernel_ms_per_step'],2), 'step ms', round(d['ms_per_step'],2))"
done
