#!/bin/bash
# Zero-copy dual-mode inputs: parity tests of the dual device mode and the
# device solves, C5 rate, the copy count per iteration, shard update-row trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_device_solve_gpu.py tests/test_fullsize_gpu.py::test_config5_window_parity -m gpu -q -x -n 4 --timeout 250 --timeout-method thread \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/tests.log | head; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000 \
  > $OUT/probe_c5.json 2> $OUT/probe_c5.err || { echo "probe failed"; tail -20 $OUT/probe_c5.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/probe_c5.json'))
for k,v in d['gpu'].items(): print(k, round(v['gpu_it_per_s'],1), {n:(s['launches'],s['device_ms'],s['call_ms']) for n,s in v['kernels'].items()})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_cp -o run -- python3 $R/scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000 > $OUT/prof_cp.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_cp.log; exit 1; }
find $OUT/prof_cp -name "*kernel_stats.csv" -exec cp {} $OUT/kstats_cp.csv \;
rm -rf $OUT/prof_cp
cut -c 1-150 $OUT/kstats_cp.csv | head -12
cd $R
for S in 1 2; do
  MILP_SHARDS=$S MILP_SMALL_FUSED=off MILP_TRACE=$OUT/trace_s$S timeout -k 10 120 python -u -c "
import sys; sys.path[:0]=['or-tools_amd','tests']
from mi_glop import abi, engine; import lp_gen
lp=lp_gen.sparse_c5_lp(2000,20000,10,97); h=engine.LpHandle(abi.default_params(use_dual_simplex=1,max_number_of_iterations=60)); h.load(lp); r=h.solve(); print('shards $S', r.problem_status, r.iterations)
" || { echo "trace run failed"; exit 1; }
done
python3 -c "
a=open('$OUT/trace_s1.device').read().splitlines(); b=open('$OUT/trace_s2.device').read().splitlines()
for i,(x,y) in enumerate(zip(a,b)):
    if x!=y: print('first diff at line', i); print(' s1', x); print(' s2', y); print(' prev', a[i-1] if i else ''); break
else: print('no diff in', min(len(a),len(b)), 'lines', len(a), len(b))"
echo done
