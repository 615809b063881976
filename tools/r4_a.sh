# Round-4 first GPU set: the new multi-GPU / voxelize-points tests, the world-1 fused (RCCL) bench
# line, then the whole GPU suite + smoke.   bash tools/r4_a.sh <outdir>
set -o pipefail
O=gpurun_out/${1:-r4a}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_round4.py tests/test_gpu_multi.py tests/test_gpu_round3.py -m gpu -x -v --timeout 400 --timeout-method thread -k "round4 or rollbuffer or adversarial or two_rank or rccl or knobs or download" > $O/pytest_new.log 2>&1 || exit 1
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --dist --steps 100 --warmup 10 --no-kernel-timing > $O/dist_n1.json 2> $O/dist_n1.err || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread --durations=15 > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
