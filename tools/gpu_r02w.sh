set -o pipefail
O=gpurun_out/r02w
mkdir -p $O
for v in nw; do
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_$v.so timeout -k 10 120 python -u -m pytest tests/test_priority_extras.py -m gpu -x -q --timeout 100 --timeout-method thread -k per_level > $O/t_$v.log 2>&1; echo "$v rc=$?"
done
