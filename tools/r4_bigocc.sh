# A/B of k_group_runs_big's register budget (GDF_BIG_OCC) on the 4K line and the C3 line.
#   bash tools/r4_bigocc.sh <outdir> <occ> ...
set -o pipefail
O=gpurun_out/${1:-r4bigocc}; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for occ in "$@"; do
  GDF_BIG_OCC=$occ timeout -k 10 120 python bench.py --steps 100 --warmup 10 --width 3840 --height 2160 --batch 1 --ring 2 --no-secondary --no-cpu-baseline > $O/4k_$occ.json 2> $O/4k_$occ.err || exit 1
  GDF_BIG_OCC=$occ timeout -k 10 180 python tools/bench_c3.py --steps 10 --json $O/c3_$occ.json > /dev/null 2>> $O/c3_$occ.err || exit 1
done
