set -o pipefail
mkdir -p gpurun_out/r02b
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 170 --timeout-method thread -k "not cfg4_full" > gpurun_out/r02b/gpu_tests.log 2>&1
echo "tests rc=$?"
tail -5 gpurun_out/r02b/gpu_tests.log
WC_LAUNCH_LOG=1 timeout -k 10 300 python -u tools/priority_bench.py --loci 1024 --cpu-loci 32 > gpurun_out/r02b/prio_cfg5.json 2> gpurun_out/r02b/prio_cfg5.err
echo "prio rc=$?"
cat gpurun_out/r02b/prio_cfg5.json
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/r02b/bench_cfg2.json 2> gpurun_out/r02b/bench_cfg2.err
echo "bench rc=$?"
cat gpurun_out/r02b/bench_cfg2.json
