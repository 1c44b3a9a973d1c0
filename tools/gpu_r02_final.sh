# Round-2 measurement set: every bench workload (with CPU baselines) + cfg2 profile passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_final3
mkdir -p $O
b() {  # tag, timeout, args...
  local tag=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail $O/$tag.err; return 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', {k: d.get(k) for k in ('loci_per_s','value','ms_per_step','kernel_ms_per_step','gpu_vs_cpu_loci','e2e_loci_per_s')}, (d.get('cpu_baseline') or {}).get('loci_per_s'))"
}
b cfg2 400 && b cfg2_latency 300 --workload cfg2-latency --steps 10 --warmup 2 && b cfg3 400 --workload cfg3 --steps 1 --warmup 1 && b cfg4 300 --workload cfg4 --steps 1 --warmup 0 && b cfg5 600 --workload cfg5 --steps 1 --warmup 0 || exit 1
bash tools/profile_round.sh r02f > $O/prof.log 2>&1 || { echo "profile failed"; tail $O/prof.log; exit 1; }
echo profile done
