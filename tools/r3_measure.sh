# Round-3 measurement set: bash tools/r3_measure.sh <outdir> (GPU suite, smoke, driver-style bench,
# 300-step line, kernel trace + separate PMC FETCH / WRITE passes of the C2 batch-8 workload, 4K
# trace, per-group traces of C3 and 4K on the diagnostic build, the C3 line)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3m}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit 1
timeout -k 10 120 python bench.py --gpus 1 --steps 300 --warmup 30 --no-secondary > $O/bench_300.json 2> $O/bench_300.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline > $O/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1 > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1 > $O/write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/t4k -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --width 3840 --height 2160 --batch 1 --ring 2 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/t4k.log 2>&1 || exit 1
timeout -k 10 150 python tools/group_trace.py --c3 256 > $O/gtrace_c3.txt 2>&1 || exit 1
timeout -k 10 120 python tools/group_trace.py 3840 2160 4 dense > $O/gtrace_4k.txt 2>&1 || exit 1
timeout -k 10 180 python tools/bench_c3.py --steps 10 --json $O/c3.json > /dev/null 2>> $O/err.log || exit 1
