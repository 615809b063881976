# The world-1 --dist (native C++ fused step over RCCL) line and its kernel trace.
# bash tools/r5/dist_trace.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5dist}; mkdir -p $O
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29521 timeout -k 10 240 python bench.py --gpus 1 --dist --steps 300 --warmup 30 --no-secondary --no-cpu-baseline > $O/dist_n1.json 2> $O/dist_n1.err || exit 1
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29523 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tdist -o run -- python bench.py --gpus 1 --dist --steps 100 --warmup 10 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/tdist.json 2> $O/tdist.err || exit 1
