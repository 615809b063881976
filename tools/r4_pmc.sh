# Round-4 counters for the C2 step (bench.py --pipeline 1: one batch in flight, rocprof averages
# comparable with the in-bench events): kernel trace, FETCH_SIZE and WRITE_SIZE passes (separate:
# the TCC slots), the SQ instruction / wait counters.   bash tools/r4_pmc.sh <outdir>
set -o pipefail
O=gpurun_out/${1:-r4pmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $B > $O/trace.json 2> $O/trace.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $B > $O/fetch.json 2> $O/fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $B > $O/write.json 2> $O/write.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/sq -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1 > $O/sq.json 2> $O/sq.err || exit 1
