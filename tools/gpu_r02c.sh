set -o pipefail
mkdir -p gpurun_out/r02c
WC_LAUNCH_LOG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_dual.py tests/test_priority_extras.py -m gpu -v --maxfail=3 --timeout 120 --timeout-method thread -k "priority or cfg4 or cfg5" > gpurun_out/r02c/prio_tests.log 2>&1
echo "prio tests rc=$?"
tail -5 gpurun_out/r02c/prio_tests.log
WC_LAUNCH_LOG=1 timeout -k 10 300 python -u tools/priority_bench.py --loci 1024 --cpu-loci 32 > gpurun_out/r02c/prio_cfg5.json 2> gpurun_out/r02c/prio_cfg5.err
echo "prio rc=$?"
cat gpurun_out/r02c/prio_cfg5.json
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 170 --timeout-method thread -k "not cfg4_full" > gpurun_out/r02c/gpu_tests.log 2>&1
echo "tests rc=$?"
tail -3 gpurun_out/r02c/gpu_tests.log
