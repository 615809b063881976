# HIP API + memory-copy trace of the world-1 --dist line (which copies / memsets a step issues).
# bash tools/r5/dist_api.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5api}; mkdir -p $O
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29525 timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/api -o run -- python bench.py --gpus 1 --dist --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/api.json 2> $O/api.err || exit 1
