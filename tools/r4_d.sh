# Run exchange (gdf_partition_runs / gdf_voxelize_runs): the multi-rank + round-4 GPU tests, the
# world-1 native --dist line, its kernel trace.   bash tools/r4_d.sh <outdir>
set -o pipefail
O=gpurun_out/${1:-r4d}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_round4.py tests/test_gpu_multi.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --dist --steps 100 --warmup 10 --no-kernel-timing --no-secondary --no-cpu-baseline > $O/dist_native.json 2> $O/dist_native.err || exit 1
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dist -o dist -- python bench.py --gpus 1 --dist --steps 100 --warmup 10 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/dist_prof.json 2> $O/dist_prof.err || exit 1
