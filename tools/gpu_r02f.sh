set -o pipefail
mkdir -p gpurun_out/r02f
timeout -k 10 60 rocprofv3 -L > gpurun_out/r02f/counters.txt 2>&1; echo "list rc=$?"
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python -u tools/phase_run.py --workload cfg3 --loci 256 --out gpurun_out/r02f/ph_cfg3 > gpurun_out/r02f/ph_cfg3.log 2>&1; echo "ph cfg3 rc=$?"
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python -u tools/phase_run.py --workload cfg5-hpc --loci 1024 --out gpurun_out/r02f/ph_cfg5 > gpurun_out/r02f/ph_cfg5.log 2>&1; echo "ph cfg5 rc=$?"
timeout -k 10 200 python -u bench.py --no-cpu --no-e2e > gpurun_out/r02f/ab_default.json 2> gpurun_out/r02f/ab_default.err; echo "ab default rc=$?"
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_split.so timeout -k 10 200 python -u bench.py --no-cpu --no-e2e > gpurun_out/r02f/ab_split.json 2> gpurun_out/r02f/ab_split.err; echo "ab split rc=$?"
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_split.so timeout -k 10 200 python -u bench.py --workload cfg3 --loci 768 --steps 1 --no-cpu > gpurun_out/r02f/ab_split_cfg3.json 2> gpurun_out/r02f/ab_split_cfg3.err; echo "ab split cfg3 rc=$?"
WC_LAUNCH_LOG=1 timeout -k 10 600 python -u bench.py --workload cfg5 --steps 1 --warmup 0 > gpurun_out/r02f/bench_cfg5.json 2> gpurun_out/r02f/bench_cfg5.err; echo "cfg5 rc=$?"
cat gpurun_out/r02f/bench_cfg5.json
