set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02p
mkdir -p $O
timeout -s KILL 200 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 --output-format csv -d $O/pcs -o run -- python3 bench.py --workload cfg3 --loci 128 --steps 1 --warmup 0 --no-cpu --no-e2e > $O/pcs_bench.json 2> $O/pcs_bench.err; echo "stochastic rc=$?"
ls -la $O/pcs 2>/dev/null
tail -5 $O/pcs_bench.err
