set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_c5
mkdir -p $O
WC_LAUNCH_LOG=1 timeout -k 10 300 python -u tools/cfg5_probe.py --loci 1024 --single 8 > $O/probe.log 2> $O/probe.err || { echo "probe failed"; tail -20 $O/probe.err; exit 1; }
cat $O/probe.log; grep -c "stream launch" $O/probe.err; grep "stream launch" $O/probe.err | tail -3
