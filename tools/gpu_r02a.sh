set -o pipefail
mkdir -p gpurun_out/r02a
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 170 --timeout-method thread -k "not cfg4_full" > gpurun_out/r02a/gpu_tests.log 2>&1
echo "tests rc=$?"
tail -5 gpurun_out/r02a/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/r02a/bench_cfg2.json 2> gpurun_out/r02a/bench_cfg2.err
echo "bench rc=$?"
cat gpurun_out/r02a/bench_cfg2.json
WC_LAUNCH_LOG=1 timeout -k 10 300 python -u tools/priority_bench.py --loci 1024 --cpu-loci 32 > gpurun_out/r02a/prio_cfg5.json 2> gpurun_out/r02a/prio_cfg5.err
echo "prio rc=$?"
cat gpurun_out/r02a/prio_cfg5.json
