set -o pipefail
O=gpurun_out/r02l
mkdir -p $O
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python -u tools/phase_run.py --workload cfg3 --loci 768 --out $O/ph_cfg3 > $O/ph_cfg3.log 2>&1; echo "ph cfg3 rc=$?"
tail -30 $O/ph_cfg3.log
WC_LAUNCH_LOG=1 timeout -k 10 300 python -u bench.py --workload cfg4 --steps 1 --warmup 0 --no-cpu > $O/bench_cfg4.json 2> $O/bench_cfg4.err; echo "cfg4 rc=$?"
grep -v amdgpu.ids $O/bench_cfg4.err | tail -20
python -c "import json; d=json.load(open('$O/bench_cfg4.json')); print('cfg4 ms', d['ms_per_step'], d['kernel_ms_per_step'])"
