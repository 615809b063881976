# The driver's C2 line (20 steps / 5 warm-up) at pipeline depths 2..4, alternating, plus the
# 300-step line per depth.  bash tools/r5/pipe_sweep.sh <outdir> <reps>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5pipe}; R=${2:-3}; mkdir -p $O
for rep in $(seq 1 $R); do
  for p in 2 3 4; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --pipeline $p --no-secondary --no-cpu-baseline > $O/p${p}_20_$rep.json 2> $O/p${p}_20_$rep.err || exit 1
  done
done
for p in 2 3 4; do
  timeout -k 10 150 python bench.py --steps 300 --warmup 30 --pipeline $p --no-secondary --no-cpu-baseline > $O/p${p}_300.json 2> $O/p${p}_300.err || exit 1
done
