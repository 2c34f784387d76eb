#!/bin/bash
# LDS-resident single-CU level runs: parity of the level plan, C5 A/B over
# the wide-level threshold.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
MILP_TRI_SYNCFREE=0 timeout -k 10 300 python -u -m pytest tests/test_device_solve_gpu.py tests/test_fullsize_gpu.py::test_config5_window_parity -m gpu -q -x -n 4 --timeout 250 --timeout-method thread \
  > $OUT/tests_levels.log 2>&1 || { echo "level-plan tests failed"; grep -E "FAILED|Error" $OUT/tests_levels.log | head; tail -30 $OUT/tests_levels.log; exit 1; }
tail -1 $OUT/tests_levels.log
MILP_TRI_SYNCFREE=0 MILP_TRI_WIDE=16000 timeout -k 10 300 python -u -m pytest tests/test_device_solve_gpu.py -m gpu -q -x -n 4 --timeout 250 --timeout-method thread \
  > $OUT/tests_levels2.log 2>&1 || { echo "level-plan (wide) tests failed"; grep -E "FAILED|Error" $OUT/tests_levels2.log | head; tail -30 $OUT/tests_levels2.log; exit 1; }
tail -1 $OUT/tests_levels2.log
timeout -k 10 400 python -u scripts/probe.py --config c5 --m 100000 --n 1000000 --warmup 20000 --steps 1000 \
  --variants "" "MILP_TRI_SYNCFREE=0" "MILP_TRI_SYNCFREE=0,MILP_TRI_WIDE=2048" "MILP_TRI_SYNCFREE=0,MILP_TRI_WIDE=4096" "MILP_TRI_SYNCFREE=0,MILP_TRI_WIDE=16000" \
  > $OUT/probe_plan.json 2> $OUT/probe_plan.err || { echo "plan probe failed"; tail -20 $OUT/probe_plan.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/probe_plan.json'))
for k,v in d['gpu'].items(): print(k, round(v['gpu_it_per_s'],1), {n:(s['launches'],s['device_ms'],s['call_ms']) for n,s in v['kernels'].items() if n.startswith('tri')})"
echo done
