# PMC FETCH_SIZE / WRITE_SIZE passes (separate runs) of the 4K single-frame line and the C3 line,
# one frame in flight, for tools/pmc_traffic.py.  bash tools/r5/pmc_secondary.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5pmc}; mkdir -p $O
B4="bench.py --width 3840 --height 2160 --batch 1 --ring 2 --pipeline 1 --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-kernel-timing"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f4k -o run --output-format csv -- python3 $B4 > $O/f4k.json 2> $O/f4k.err || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w4k -o run --output-format csv -- python3 $B4 > $O/w4k.json 2> $O/w4k.err || exit 1
BC="tools/bench_c3.py --steps 3 --profile-steps 1"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fc3 -o run --output-format csv -- python3 $BC > $O/fc3.out 2> $O/fc3.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/wc3 -o run --output-format csv -- python3 $BC > $O/wc3.out 2> $O/wc3.err || exit 1
