#!/bin/bash
# rocprofv3 evidence for the bench's rooflines, one workload per process so
# that per-kernel-id byte counts are not mixed:
#   C2: scripts/probe.py --config c2        -> gpurun_out/prof_c2/{trace,fetch,write}
#   C5: scripts/probe.py --config c5        -> gpurun_out/prof_c5/{trace,fetch,write}
#   C4M: ta041-shaped mid-size batch (50x10, 16 children, 1 worker)
#   C4: scripts/probe_batch.py (256 children, 1 worker: rocprofv3 crashed
#       under 8 concurrent worker threads) -> gpurun_out/prof_c4/...
# Kernel trace + stats in one run; FETCH_SIZE and WRITE_SIZE in runs of their
# own (MI355X_MICROARCH.md HBM recipe). Each workload is summarised right
# after its passes (scripts/profile_summary.py) and its raw traces, which
# exceed the 64 MiB merge limit, are deleted.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
C2="python3 $R/scripts/probe.py --config c2 --warmup 3 --steps 64"
C4="python3 $R/scripts/probe_batch.py --lps 256 --workers 1"
C4M="python3 $R/scripts/probe_batch.py --jobs 50 --machines 10 --lps 16 --workers 1"
C5="python3 $R/scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup ${C5_WARMUP:-20000} --steps ${C5_STEPS:-1000}"
for W in ${WORKLOADS:-c2 c5}; do
  if [ "$W" = c2 ]; then CMD=$C2; elif [ "$W" = c4 ]; then CMD=$C4; elif [ "$W" = c4m ]; then CMD=$C4M; else CMD=$C5; fi
  P=$OUT/prof_$W
  mkdir -p $P
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $P/trace -o run -- $CMD > $P/trace.log 2>&1 || { echo "$W trace failed"; tail -20 $P/trace.log; rm -rf $P; exit 1; }
  echo "$W trace done $(date +%T)"
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $P/fetch -o run -- $CMD > $P/fetch.log 2>&1 || { echo "$W fetch failed"; tail -20 $P/fetch.log; rm -rf $P; exit 1; }
  echo "$W fetch done $(date +%T)"
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $P/write -o run -- $CMD > $P/write.log 2>&1 || { echo "$W write failed"; tail -20 $P/write.log; rm -rf $P; exit 1; }
  echo "$W write done $(date +%T)"
  PROFILE_OUT_ROOT=$OUT/profiles python3 $R/scripts/profile_summary.py $P ${TAG:-r01}_$W $W > /dev/null || { echo "summary $W failed"; rm -rf $P; exit 1; }
  cp $P/*.log $OUT/profiles/${TAG:-r01}_$W/ 2>/dev/null
  rm -rf $P
done
ls -R $OUT/profiles
