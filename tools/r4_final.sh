# Round-4 measurement set: bash tools/r4_final.sh <outdir> - GPU suite, smoke, the default line
# (python bench.py: 300 / 30, every secondary), the short line (20 / 5), the 300-step line, the world-1 --dist (native) line, the kernel trace
# of the C2 step with one batch in flight, PMC FETCH / WRITE / SQ passes of it, the 4K trace, the
# world-1 --dist trace, the C3 line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread --durations=15 > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit 1
timeout -k 10 150 python bench.py --gpus 1 --steps 300 --warmup 30 --no-secondary > $O/bench_300.json 2> $O/bench_300.err || exit 1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --dist --steps 100 --warmup 10 --no-secondary --no-cpu-baseline > $O/dist_n1.json 2> $O/dist_n1.err || exit 1
B="bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B > $O/trace.json 2> $O/trace.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $B > $O/fetch.json 2> $O/fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $B > $O/write.json 2> $O/write.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/sq -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1 > $O/sq.json 2> $O/sq.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/t4k -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --width 3840 --height 2160 --batch 1 --ring 2 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/t4k.json 2> $O/t4k.err || exit 1
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tdist -o run -- python bench.py --gpus 1 --dist --steps 100 --warmup 10 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/tdist.json 2> $O/tdist.err || exit 1
timeout -k 10 180 python tools/bench_c3.py --steps 10 --json $O/c3.json > /dev/null 2>> $O/c3.err || exit 1
