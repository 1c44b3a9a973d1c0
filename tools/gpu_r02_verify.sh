# Round-2 re-entry verification on the GPU box: GPU parity suite, smoke, cfg2 bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_verify
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo "bench failed"; tail -20 $O/bench_cfg2.err; exit 1; }
cat $O/bench_cfg2.json
