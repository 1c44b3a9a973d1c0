# Round-2 closing check, as the driver runs it: GPU parity suite, smoke, default bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_last
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print({k: d.get(k) for k in ('loci_per_s','value','ms_per_step','ms_per_step_median','kernel_ms_per_step','gpu_vs_cpu_loci','e2e_loci_per_s','e2e_vs_cpu_loci')}); print(d['roofline']['achieved'], d['roofline']['frac'], d['roofline']['pmc_source'], d['cpu_baseline']['loci_per_s'], d['cpu_baseline']['cores'])"
