# cfg5 bulk throughput vs dual-engine occupancy (LDS budget / register budget)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_occ
mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" WC_LAUNCH_LOG=1 timeout -k 10 300 python -u bench.py --workload cfg5 --loci 4096 --steps 1 --warmup 0 --no-cpu > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail $O/$tag.err; return 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag cfg5 4096 loci/s', round(d['loci_per_s'],1))"; grep "stream launch" $O/$tag.err | head -2
}
run w3lds24 WC_DUAL_LDS_KB=24 WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_w3.so && run base WC_NARROW=2
