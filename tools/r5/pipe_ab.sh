# Pipeline-depth sweep, abtree/<A> against this tree, C2 300-step lines.
# bash tools/r5/pipe_ab.sh <outdir> <A> <depth>...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5pipe}; A=${2:-r5p}; shift 2; mkdir -p $O
for d in "$@"; do
  (cd abtree/$A && timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline --pipeline $d) > $O/a_p$d.json 2> $O/a_p$d.err || exit 1
  timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline --pipeline $d > $O/b_p$d.json 2> $O/b_p$d.err || exit 1
done
