set -o pipefail
mkdir -p gpurun_out/r02h
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_single.py tests/test_gpu_fullsize.py -m gpu -v --maxfail=3 --timeout 170 --timeout-method thread -k "not cfg4_full" > gpurun_out/r02h/tests.log 2>&1
echo "tests rc=$?"
tail -3 gpurun_out/r02h/tests.log
timeout -k 10 200 python -u bench.py --no-cpu > gpurun_out/r02h/bench_cfg2.json 2> gpurun_out/r02h/bench_cfg2.err; echo "bench rc=$?"
cat gpurun_out/r02h/bench_cfg2.json
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r02h/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e > gpurun_out/r02h/write_bench.json; echo "write rc=$?"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/r02h/lds -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e > gpurun_out/r02h/lds_bench.json; echo "lds rc=$?"
