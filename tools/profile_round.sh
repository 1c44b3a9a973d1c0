#!/bin/bash
# Profiles one bench workload on the GPU box (run through gpurun):
#   kt     kernel trace + stats (per-kernel durations)
#   fetch  PMC FETCH_SIZE            } separate passes: TCC slots
#   write  PMC WRITE_SIZE            }
#   sq1    PMC issue view: wave cycles, busy/wait split, VALU/SALU instructions
#   sq2    PMC LDS view: LDS instructions, bank conflicts, LDS issue stalls, memory instructions
# Every pass is its own timeout-bounded run. Outputs under gpurun_out/prof_<tag>/;
# tools/pmc_summary.py condenses them into profiles/.
#   bash tools/profile_round.sh <tag> [bench args...]
# PASSES="kt fetch write" limits the passes (default: kt fetch write sq1; sq2
# and tcc on request: an 8-counter SQ pass of derived LDS/VMEM counters was
# refused on the box in round 6, so sq2 holds 4 counters now). The default
# bench line also runs the cfg5 leg: give cfg2 runs --cfg5-loci 0.
set -e
PASSES=${PASSES:-"kt fetch write sq1"}
on() { case " $PASSES " in *" $1 "*) return 0;; esac; return 1; }
TAG=${1:-r02}
shift || true
ARGS="$@"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
# heartbeat: a pass writes nothing until it ends (a 10,000-locus cfg5 pass runs
# minutes), and gpurun takes 3 silent minutes for a hang
( while sleep 30; do date >> $OUT/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if on kt; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e $ARGS > $OUT/kt_bench.json
echo "kt done"
fi
if on fetch; then
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e $ARGS > $OUT/fetch_bench.json
echo "fetch done"
fi
if on write; then
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e $ARGS > $OUT/write_bench.json
echo "write done"
fi
if on sq1; then
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $OUT/sq1 -o run -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e $ARGS > $OUT/sq1_bench.json
echo "sq1 done"
fi
if on sq2; then
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  --output-format csv -d $OUT/sq2 -o run -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e $ARGS > $OUT/sq2_bench.json
echo "sq2 done"
fi
if on tcc; then
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum \
  --output-format csv -d $OUT/tcc -o run -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e $ARGS > $OUT/tcc_bench.json
echo "profile $TAG done"
fi
