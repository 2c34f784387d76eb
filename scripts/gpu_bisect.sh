# Runs one GPU test under several engine switches, one process each; stops
# at the first run that neither passes nor fails cleanly.
set -o pipefail
T=${T:-"tests/test_device_solve_gpu.py::test_device_u_solve_with_async_tau_and_device_dual"}
for V in ${VARIANTS:-"MILP_TRI_SYNCFREE=0"}; do
  echo "== $V $(date +%T)"
  env $V MILP_WATCHDOG_S=${WATCHDOG:-15} timeout -k 10 ${LIMIT:-100} python -u -X faulthandler -m pytest $T -x -s -v --timeout 80 --timeout-method thread > gpurun_out/bisect_${V%%=*}.log 2>&1
  rc=$?
  echo "rc=$rc"; grep -E "PASSED|FAILED|Timeout|Error|watchdog" gpurun_out/bisect_${V%%=*}.log | head -12
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then break; fi
done
