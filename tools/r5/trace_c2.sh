# C2 kernel traces: 3 batches in flight (the bench line's pipeline) and 1 in flight, plus the A/B of
# this tree against abtree/r4.  bash tools/r5/trace_c2.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5t}; mkdir -p $O
B="bench.py --steps 100 --warmup 10 --no-secondary --no-cpu-baseline --no-kernel-timing"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/p3 -o run --output-format csv -- python3 $B > $O/p3.json 2> $O/p3.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/p1 -o run --output-format csv -- python3 $B --pipeline 1 > $O/p1.json 2> $O/p1.err || exit 1
for i in 1 2; do
  (cd abtree/r4 && timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline) > $O/a$i.json 2> $O/a$i.err || exit 1
  timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline > $O/b$i.json 2> $O/b$i.err || exit 1
done
