#!/bin/bash
# Round 4: kernel trace of config 5's late window (probe, 300 iterations
# from 20 020), to split a U solve into its launches and the gaps between.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r04_c5trace
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python3 -u $R/scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20020 --steps 300 \
  > $OUT/probe.json 2> $OUT/probe.err || exit 1
cd $R
python3 scripts/trace_window.py $OUT/trace $OUT/probe.json > $OUT/window.txt || exit 1
cat $OUT/window.txt | head -60
