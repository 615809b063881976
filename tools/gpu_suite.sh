# Full GPU suite + smoke: bash tools/gpu_suite.sh <outdir>
set -o pipefail
out=gpurun_out/${1:-suite}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > $out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
