# Round-5 baseline: the default line, the 300-step C2 line, the C2 kernel trace (one batch in
# flight), the 4K trace, the C3 line.  bash tools/r5/base.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5base}; mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 150 python bench.py --gpus 1 --steps 300 --warmup 30 --no-secondary > $O/bench_300.json 2> $O/bench_300.err || exit 1
B="bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B > $O/trace.json 2> $O/trace.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/t4k -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --width 3840 --height 2160 --batch 1 --ring 2 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/t4k.json 2> $O/t4k.err || exit 1
timeout -k 10 180 python tools/bench_c3.py --steps 10 --json $O/c3.json > /dev/null 2>> $O/c3.err || exit 1
