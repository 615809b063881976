# k_mask A/B: abtree/<A> against this tree - a parity subset on this tree, then per tree and rep
# the C2 line (300 steps) and a kernel-trace summary of a 100-step C2 run, alternating.
# bash tools/r5/mask_ab.sh <outdir> <A> <reps>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5mask}; A=${2:-base}; R=${3:-2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "batch8 or mask or smoke or adversarial" > $O/pytest_subset.log 2>&1 || exit 1
for rep in $(seq 1 $R); do
  for v in a b; do
    if [ $v = a ]; then D=abtree/$A; else D=.; fi
    (cd $D && timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline) > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 1
    (cd $D && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof_${v}_$rep -o run -- python bench.py --steps 100 --warmup 10 --no-secondary --no-cpu-baseline) > $O/prof_${v}_$rep.log 2>&1 || exit 1
  done
done
