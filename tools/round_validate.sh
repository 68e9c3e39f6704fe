# Full GPU test suite, smoke, the default bench line + rocprof of its roofline op (tools/roofline_profile.sh)
set -euo pipefail
mkdir -p gpurun_out/v4
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v4/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v4/smoke.log 2>&1
bash tools/roofline_profile.sh
