# Round-4 measurement pass 1: the driver-style bench line, a kernel trace of the C2 step (one
# batch in flight, so rocprof averages compare with the in-bench events), and a kernel trace of the
# world-1 fused (RCCL) step.   bash tools/r4_b.sh <outdir>
set -o pipefail
O=gpurun_out/${1:-r4b}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_round4.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python bench.py --steps 200 --warmup 20 --no-secondary --no-cpu-baseline --pipeline 1 > $O/c2_p1.json 2> $O/c2_p1.err || exit 1
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dist -o dist -- python bench.py --gpus 1 --dist --steps 100 --warmup 10 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/dist.json 2> $O/dist.err || exit 1
