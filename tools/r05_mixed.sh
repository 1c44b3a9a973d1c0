#!/bin/bash
# GPU box: GPU suites with the wave engine as the dual default (mixed R
# kernel), PMC views of the wave kernel on the 5949 full-read level, the
# 2000-locus cfg5 per-locus latency
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dual.py tests/test_gpu_builds.py tests/test_gpu_service.py tests/test_priority_extras.py tests/test_gpu_offsets.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
C2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAVES"
k=0
for C in "$C1" "$C2"; do
  k=$((k+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/pmc$k -o run -- python3 tools/one_sub.py --workload cfg5-full --seed 5949 > $O/pmc$k.json 2>&1 || exit 1
done
timeout -k 10 300 python3 -u tools/cfg5_lat.py --loci 2000 --out $O/lat > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
grep -v amdgpu.ids $O/lat.log | head -8
