#!/bin/bash
# SQ counters of the device dual segments on a config-4 batch (64 children,
# MILP_SDUAL_POOL=0: one single-workgroup launch per segment, so a dispatch's
# counters are one LP's segment): instruction fetch, where a wave's cycles go
# (waiting vs issuing) and the instruction mix. One --pmc pass per run (the
# per-block counter limits of MI355X_MICROARCH.md); a failing pass ends the
# session.   scripts/pmc_sdual.sh OUT_DIR
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -o "SQC\?_[A-Z_0-9]*" $OUT/avail.txt | sort -u > $OUT/sq_counters.txt || true
P1="SQ_IFETCH SQ_IFETCH_LEVEL SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P3="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
n=1
for P in "$P1" "$P2" "$P3"; do
  Q=""
  for c in $P; do if grep -qx "$c" $OUT/sq_counters.txt; then Q="$Q $c"; else echo "missing $c"; fi; done
  [ -n "$Q" ] || { echo "pass $n skipped"; n=$((n+1)); continue; }
  MILP_SDUAL_POOL=0 MILP_CRASH_REPORT=1 MILP_DEVICE_RESET_AT_EXIT=1 timeout -s KILL 240 rocprofv3 --pmc $Q -d $OUT/p$n -o p$n \
    --output-format csv -- python3 $R/scripts/probe_batch.py --node --lps 64 --workers 64 \
    > $OUT/p$n.log 2>&1
  rc=$?; echo "pass $n rc=$rc"
  [ $rc -eq 0 ] || { python3 $R/scripts/pmc_sum.py $OUT > $OUT/summary.txt 2>&1; exit $rc; }
  n=$((n+1))
done
python3 $R/scripts/pmc_sum.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
