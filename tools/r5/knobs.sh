# Knob sweep on one box, alternating: every variant (env assignments, "base" = none) twice, the
# C2 300-step line (+ extra bench args).  bash tools/r5/knobs.sh <outdir> "<extra args>" v1 v2 ...
# e.g. bash tools/r5/knobs.sh r5k "" base "GDF_SORT_BLOCKS=256" "GDF_SORT_BLOCKS=256 GDF_GROUP_BLOCKS=512"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5k}; X=$2; shift 2; mkdir -p $O
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    if [ "$v" = base ]; then E=""; else E="$v"; fi
    env $E timeout -k 10 150 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline $X > $O/v${i}_r$rep.json 2> $O/v${i}_r$rep.err || exit 1
    echo "v$i: $v" > $O/v${i}.name
  done
done
