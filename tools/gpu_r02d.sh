set -o pipefail
mkdir -p gpurun_out/r02d
WC_LAUNCH_LOG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_dual.py tests/test_priority_extras.py tests/test_gpu_single.py tests/test_gpu_dwfa.py -m gpu -v --maxfail=3 --timeout 120 --timeout-method thread > gpurun_out/r02d/tests1.log 2>&1
echo "tests1 rc=$?"
tail -5 gpurun_out/r02d/tests1.log
WC_LAUNCH_LOG=1 timeout -k 10 300 python -u tools/priority_bench.py --loci 1024 --cpu-loci 32 > gpurun_out/r02d/prio_cfg5.json 2> gpurun_out/r02d/prio_cfg5.err
echo "prio rc=$?"
cat gpurun_out/r02d/prio_cfg5.json
