# Kernel trace of the C2 line at pipeline depth 4 with 8 HIP hardware queues (100 steps).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5ptrace8}; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
for p in 4 3; do
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/p$p -o run -- python bench.py --steps 100 --warmup 10 --pipeline $p --no-secondary --no-cpu-baseline > $O/p$p.log 2>&1 || exit 1
done
