# A/B of the k_sel tile shape (GDF_SEL_SHAPE "segs,threads") on the C3 line.
#   bash tools/r4_selshape.sh <outdir> <shape> ...   ("default" = the engine's choice)
set -o pipefail
O=gpurun_out/${1:-r4sel}; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for sh in "$@"; do
  tag=${sh/,/x}
  if [ "$sh" = default ]; then
    timeout -k 10 180 python tools/bench_c3.py --steps 10 --json $O/c3_$tag.json > /dev/null 2>> $O/c3_$tag.err || exit 1
  else
    GDF_SEL_SHAPE=$sh timeout -k 10 180 python tools/bench_c3.py --steps 10 --json $O/c3_$tag.json > /dev/null 2>> $O/c3_$tag.err || exit 1
  fi
done
