set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "full_row or full_and_partial or dense" > gpurun_out/gpu_tests_fr.log 2>&1 || { echo "full-row tests failed"; tail -60 gpurun_out/gpu_tests_fr.log; exit 1; }
tail -1 gpurun_out/gpu_tests_fr.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
SKIP_C5=1 bash scripts/gpu_phase.sh
