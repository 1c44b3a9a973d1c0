#!/bin/bash
# PMC instruction mix of one cfg5-hpc sub-problem alone, old engine vs wave engine
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
for eng in 0 1; do
  WC_WAVE=$eng timeout -k 10 120 python3 tools/one_sub.py --seed 48 > $O/time_$eng.json || exit 1
  WC_WAVE=$eng timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_ANY --output-format csv -d $O/pmc_$eng -o run -- python3 tools/one_sub.py --seed 48 > $O/pmc_$eng.json || exit 1
done
echo done
