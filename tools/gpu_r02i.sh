set -o pipefail
mkdir -p gpurun_out/r02i
timeout -k 10 400 python -u -m pytest tests/test_gpu_dual.py tests/test_priority_extras.py tests/test_gpu_fullsize.py tests/test_gpu_offsets.py -m gpu -v --maxfail=3 --timeout 170 --timeout-method thread -k "not cfg4_full" > gpurun_out/r02i/tests.log 2>&1
echo "tests rc=$?"
tail -3 gpurun_out/r02i/tests.log
timeout -k 10 200 python -u bench.py --workload cfg3 --loci 768 --steps 1 --warmup 1 --no-cpu > gpurun_out/r02i/bench_cfg3.json 2> gpurun_out/r02i/bench_cfg3.err; echo "cfg3 rc=$?"
python -c "import json; d=json.load(open('gpurun_out/r02i/bench_cfg3.json')); print('cfg3 loci/s', d['loci_per_s'], 'kernel ms', d['kernel_ms_per_step'])"
WC_LAUNCH_LOG=1 timeout -k 10 300 python -u tools/priority_bench.py --loci 1024 --cpu-loci 16 > gpurun_out/r02i/prio_cfg5.json 2> gpurun_out/r02i/prio_cfg5.err; echo "prio rc=$?"
cat gpurun_out/r02i/prio_cfg5.json
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python -u tools/phase_run.py --workload cfg5-hpc --loci 1024 --out gpurun_out/r02i/ph_cfg5 > gpurun_out/r02i/ph_cfg5.log 2>&1; echo "ph cfg5 rc=$?"
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python -u tools/phase_run.py --workload cfg3 --loci 256 --out gpurun_out/r02i/ph_cfg3 > gpurun_out/r02i/ph_cfg3.log 2>&1; echo "ph cfg3 rc=$?"
