# The C++ multi-rank step through the in-process transport on one GPU (+ the RCCL world-1 form and
# the round-5 tests), then bench lines: the launcher with gloo ranks, the local transport.
set -o pipefail
out=gpurun_out/${1:-r5a}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_local_world.py tests/test_gpu_round5.py -v --timeout 400 --timeout-method thread --durations=10 > $out/t.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py -k world1 -v --timeout 200 --timeout-method thread > $out/t1.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 --no-kernel-timing > $out/gloo2.json 2> $out/gloo2.err && \
timeout -k 10 300 python bench.py --gpus 4 --transport local --steps 100 --warmup 10 > $out/local4.json 2> $out/local4.err
