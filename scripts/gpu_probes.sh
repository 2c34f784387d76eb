set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 200 python -u $R/scripts/probe_batch.py --lps 512 --workers 1 8 16 > $OUT/probe_on.json 2> $OUT/probe_on.err || exit 1
timeout -k 10 300 python -u $R/scripts/probe_c3.py --workers 1 8 16 > $OUT/probe_c3.json 2> $OUT/probe_c3.err || exit 1
cat $OUT/probe_on.err $OUT/probe_c3.err
