set -o pipefail
mkdir -p gpurun_out/r02e
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 170 --timeout-method thread -k "not cfg4_full" > gpurun_out/r02e/gpu_tests.log 2>&1
echo "tests rc=$?"
tail -3 gpurun_out/r02e/gpu_tests.log
timeout -k 10 300 python -u bench.py --workload cfg3 --loci 768 --steps 1 --warmup 1 > gpurun_out/r02e/bench_cfg3.json 2> gpurun_out/r02e/bench_cfg3.err
echo "cfg3 rc=$?"
cat gpurun_out/r02e/bench_cfg3.json
WC_LAUNCH_LOG=1 timeout -k 10 400 python -u bench.py --workload cfg5 --steps 1 --warmup 0 > gpurun_out/r02e/bench_cfg5.json 2> gpurun_out/r02e/bench_cfg5.err
echo "cfg5 rc=$?"
cat gpurun_out/r02e/bench_cfg5.json
timeout -k 10 300 python -u bench.py > gpurun_out/r02e/bench_cfg2.json 2> gpurun_out/r02e/bench_cfg2.err
echo "cfg2 rc=$?"
cat gpurun_out/r02e/bench_cfg2.json
