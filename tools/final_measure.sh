set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/final5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit 1
timeout -k 10 200 python bench.py --gpus 1 --steps 300 --warmup 30 --no-secondary > $O/bench_300.json 2> $O/bench_300.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1 > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1 > $O/write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/sq -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/sq.log 2>&1 || exit 1
