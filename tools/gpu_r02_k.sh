set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_k
mkdir -p $O
WC_LAUNCH_LOG=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-e2e > $O/cfg2_def.json 2> $O/cfg2_def.err || { echo "def failed"; exit 1; }
grep "launch sides" $O/cfg2_def.err | tail -1
python -c "import json; d=json.load(open('$O/cfg2_def.json')); print('default kernel ms', round(d['kernel_ms_per_step'],2))"
for k in 40; do
  WC_CHAIN=$k timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-e2e > $O/cfg2_$k.json 2> $O/cfg2_$k.err || { echo "k$k failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg2_$k.json')); print('K=$k kernel ms', round(d['kernel_ms_per_step'],2))"
done
