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
grep -o "SQ_[A-Z_0-9]*" $OUT/avail.txt | sort -u > $OUT/sq_counters.txt || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
n=1
for P in "$P1" "$P2"; do
  ok=1
  for c in $P; do grep -qx "$c" $OUT/sq_counters.txt || { echo "missing $c"; ok=0; }; done
  [ $ok -eq 1 ] || { echo "pass $n skipped"; n=$((n+1)); continue; }
  MILP_SDUAL_POOL=0 timeout -s KILL 240 rocprofv3 --pmc $P -d $OUT/p$n -o p$n --output-format csv -- \
    python3 $R/scripts/probe_batch.py --node --lps 64 --workers 64 > $OUT/p$n.log 2>&1
  rc=$?; echo "pass $n rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  n=$((n+1))
done
find $OUT -name "*counter_collection*" | head
