# Kernel trace + stats of the C2 line with one batch in flight (this tree).  bash tools/r5/trace1.sh <outdir> [env...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5t1}; shift; mkdir -p $O
for kv in "$@"; do export "$kv"; done
B="bench.py --steps 100 --warmup 10 --no-secondary --no-cpu-baseline --no-kernel-timing"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/p1 -o run --output-format csv -- python3 $B --pipeline 1 > $O/p1.json 2> $O/p1.err
