#!/bin/bash
# Vector-memory pipeline view of the one-wave dual engine (GPU box): two PMC
# passes (SQ latency levels; TA/TCP busy and stalls) on a throughput-bound
# batch of cfg5 loci of at most 64 reads and on one sub-problem alone.
#   bash tools/pmc_vmem.sh <out dir under gpurun_out>
set -e
out=${1:-gpurun_out/vmem}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
A="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
B="TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TCP_PENDING_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
for w in batch one; do
  if [ $w = batch ]; then cmd="python3 -u $R/tools/cfg5_small.py --loci 6000"; else cmd="python3 -u $R/tools/one_sub.py --workload cfg5-full --seed 5 --reps 1"; fi
  timeout -s KILL 200 rocprofv3 --pmc $A -d $R/$out/${w}_a -o pmc -- $cmd > $R/$out/${w}_a.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc $B -d $R/$out/${w}_b -o pmc -- $cmd > $R/$out/${w}_b.log 2>&1
done
