#!/bin/bash
# Round 4: SQ counters of the sdual pool kernel on a config-4 batch (256
# children; MILP_SDUAL_POOL=0: one single-workgroup launch per segment, so
# a dispatch's counters are one LP's segment): where a wave's cycles go (waiting on memory vs
# issuing), and the instruction mix. Each --pmc pass is its own run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -o "SQC\?_[A-Z_0-9]*" $OUT/avail.txt | sort -u > $OUT/sq_counters.txt || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
# Instruction fetch: the segment kernel is ~250 KB of code against a 64 KB
# instruction cache shared by two CUs.
P3="SQ_IFETCH SQ_IFETCH_LEVEL SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
n=1
for P in "$P3" "$P1" "$P2"; do
  ok=1
  Q=""
  for c in $P; do if grep -qx "$c" $OUT/sq_counters.txt; then Q="$Q $c"; else echo "missing $c"; fi; done
  P=$Q
  [ -n "$P" ] || { echo "pass $n skipped"; n=$((n+1)); continue; }
  MILP_SDUAL_POOL=0 timeout -s KILL 240 rocprofv3 --pmc $P -d $OUT/p$n -o p$n --output-format csv -- \
    python3 $R/scripts/probe_batch.py --node --lps 64 --workers 64 > $OUT/p$n.log 2>&1
  rc=$?; echo "pass $n rc=$rc"
  # A failing pass (rocprofv3 has exited 139 at teardown after writing its
  # counters) ends the GPU work of this call.
  [ $rc -eq 0 ] || { python3 $R/scripts/pmc_sum.py $OUT > $OUT/summary.txt 2>&1; exit $rc; }
  n=$((n+1))
done
python3 $R/scripts/pmc_sum.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
