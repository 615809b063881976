# Group-first as the default: the GPU suite, smoke, the C2 300-step line and the C3 line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5final6}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline > $O/bench_300.json 2> $O/bench_300.err || exit 1
timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/bench_20_5.json 2> $O/bench_20_5.err || exit 1
timeout -k 10 200 python tools/bench_c3.py --steps 10 --json $O/c3.json > /dev/null 2>> $O/c3.err || exit 1
