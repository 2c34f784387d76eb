#!/bin/bash
# Same-box C5 A/B: the tree in _old/ (previous commit, built in-tree) against
# this tree, alternated; C5 section only.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
for rep in 1 2; do
  for t in _old .; do
    cd $R/$t
    timeout -k 10 240 python -u bench.py --no-cpu --no-c2 --no-c3 --batch-lps 16 --batch-workers 16 > $OUT/c5ab.json 2> $OUT/c5ab.err || { echo "$t failed"; tail -20 $OUT/c5ab.err; exit 1; }
    python -c "import json;d=json.loads(open('$OUT/c5ab.json').read().strip().splitlines()[-1]);print('$t', round(d['value']), d['host_ms_per_step'], d['device_call_ms_per_step'])"
  done
done
echo done
