#!/bin/bash
# rocprofv3 evidence for the bench's rooflines, one workload per process so
# that per-kernel-id byte counts are not mixed:
#   C2: bench.py's config-2 section only   -> gpurun_out/prof_c2/{trace,fetch,write}
#   C5: scripts/probe.py --config c5        -> gpurun_out/prof_c5/{trace,fetch,write}
#   C4: scripts/probe_batch.py (512 children, 8 workers) -> gpurun_out/prof_c4/...
# Kernel trace + stats in one run; FETCH_SIZE and WRITE_SIZE in runs of their
# own (MI355X_MICROARCH.md HBM recipe). Summarise afterwards with
#   python scripts/profile_summary.py gpurun_out/prof_c2 <tag> c2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
C2="python3 $R/bench.py --no-cpu --no-c5 --no-c3 --batch-lps 0"
C4="python3 $R/scripts/probe_batch.py --lps 512 --workers 8"
C5="python3 $R/scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup ${C5_WARMUP:-20000} --steps ${C5_STEPS:-1000}"
for W in ${WORKLOADS:-c2 c5}; do
  if [ "$W" = c2 ]; then CMD=$C2; elif [ "$W" = c4 ]; then CMD=$C4; else CMD=$C5; fi
  P=$OUT/prof_$W
  mkdir -p $P
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $P/trace -o run -- $CMD > $P/trace.log 2>&1 || { echo "$W trace failed"; tail -20 $P/trace.log; exit 1; }
  echo "$W trace done $(date +%T)"
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $P/fetch -o run -- $CMD > $P/fetch.log 2>&1 || { echo "$W fetch failed"; tail -20 $P/fetch.log; exit 1; }
  echo "$W fetch done $(date +%T)"
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $P/write -o run -- $CMD > $P/write.log 2>&1 || { echo "$W write failed"; tail -20 $P/write.log; exit 1; }
  echo "$W write done $(date +%T)"
done
# Summaries come back under gpurun_out/profiles/ (the raw traces exceed the
# 64 MiB merge limit and are deleted here).
for W in ${WORKLOADS:-c2 c5}; do
  PROFILE_OUT_ROOT=$OUT/profiles python3 $R/scripts/profile_summary.py $OUT/prof_$W ${TAG:-r01}_$W $W > /dev/null || { echo "summary $W failed"; exit 1; }
  cp $OUT/prof_$W/*.log $OUT/profiles/${TAG:-r01}_$W/ 2>/dev/null
  rm -rf $OUT/prof_$W
done
ls -R $OUT/profiles
