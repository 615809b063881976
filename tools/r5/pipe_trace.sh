# Kernel traces of the C2 line at pipeline depths 3 and 4 (100 steps).  bash tools/r5/pipe_trace.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5ptrace}; mkdir -p $O
for p in 3 4; do
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/p$p -o run -- python bench.py --steps 100 --warmup 10 --pipeline $p --no-secondary --no-cpu-baseline > $O/p$p.log 2>&1 || exit 1
done
