# A/B of tuning knobs on the C2 line (each a separate process; the bench's own timing).
#   bash tools/r4_sweep.sh <outdir> "<label>:<ENV=V ...>[|<extra bench args>]" ...
set -o pipefail
O=gpurun_out/${1:-r4sweep}; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for spec in "$@"; do
  label=${spec%%:*}; rest=${spec#*:}
  envs=${rest%%|*}; extra=""
  [ "$rest" != "$envs" ] && extra=${rest#*|}
  for rep in 1 2; do
    env $envs timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-secondary --no-cpu-baseline --no-kernel-timing $extra > $O/$label.$rep.json 2> $O/$label.$rep.err || exit 1
  done
done
