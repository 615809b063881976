# HIP hardware queues per process (GPU_MAX_HW_QUEUES, the image's default 4) against the pipeline
# depth on the C2 line: 20-step (the driver's) and 300-step lines, alternating.
# bash tools/r5/queue_sweep.sh <outdir> <reps>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5queue}; R=${2:-2}; mkdir -p $O
for rep in $(seq 1 $R); do
  for cfg in 4:3 8:3 8:4 8:5 8:6; do
    q=${cfg%%:*}; p=${cfg##*:}
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --steps 20 --warmup 5 --pipeline $p --no-secondary --no-cpu-baseline > $O/q${q}p${p}_20_$rep.json 2> $O/q${q}p${p}_20_$rep.err || exit 1
  done
done
for cfg in 4:3 8:3 8:4 8:5 8:6; do
  q=${cfg%%:*}; p=${cfg##*:}
  GPU_MAX_HW_QUEUES=$q timeout -k 10 150 python bench.py --steps 300 --warmup 30 --pipeline $p --no-secondary --no-cpu-baseline > $O/q${q}p${p}_300.json 2> $O/q${q}p${p}_300.err || exit 1
done
