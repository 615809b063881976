# Native fused rank (gdf_fused_*): RCCL world-1 tests, then the world-1 --dist bench line (native
# and python) and a kernel trace of the native step.   bash tools/r4_c.sh <outdir>
set -o pipefail
O=gpurun_out/${1:-r4c}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -m gpu -x -v --timeout 200 --timeout-method thread -k "rccl" > $O/pytest_rccl.log 2>&1 || exit 1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --dist --steps 100 --warmup 10 --no-kernel-timing --no-secondary --no-cpu-baseline > $O/dist_native.json 2> $O/dist_native.err || exit 1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --dist --steps 100 --warmup 10 --no-kernel-timing --no-secondary --no-cpu-baseline --fused-impl python > $O/dist_python.json 2> $O/dist_python.err || exit 1
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dist -o dist -- python bench.py --gpus 1 --dist --steps 100 --warmup 10 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/dist_prof.json 2> $O/dist_prof.err || exit 1
