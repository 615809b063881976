# A/B on one box: abtree/<A> (an older tree with its built library) against this tree, alternating,
# C2 300-step lines.  bash tools/r5/ab.sh <outdir> <A> [extra bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5ab}; A=${2:-r4}; shift 2; mkdir -p $O
for i in 1 2 3; do
  (cd abtree/$A && timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline "$@") > $O/a$i.json 2> $O/a$i.err || exit 1
  timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline "$@" > $O/b$i.json 2> $O/b$i.err || exit 1
done
