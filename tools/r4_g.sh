# Emit partition (GDF_EMIT_PART=1): the multi-rank + round-4 GPU tests with it, then the world-1
# native --dist line with and without it, and a kernel trace with it.   bash tools/r4_g.sh <outdir>
set -o pipefail
O=gpurun_out/${1:-r4g}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export GDF_EMIT_PART=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_round4.py tests/test_gpu_multi.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --dist --steps 100 --warmup 10 --no-kernel-timing --no-secondary --no-cpu-baseline > $O/dist_emit.json 2> $O/dist_emit.err || exit 1
env -u GDF_EMIT_PART timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --dist --steps 100 --warmup 10 --no-kernel-timing --no-secondary --no-cpu-baseline > $O/dist_pass.json 2> $O/dist_pass.err || exit 1
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dist -o dist -- python bench.py --gpus 1 --dist --steps 100 --warmup 10 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/dist_prof.json 2> $O/dist_prof.err || exit 1
