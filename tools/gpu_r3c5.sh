set -o pipefail
bash tools/gpu_suite.sh r3c5 && bash tools/gpu_perf_groups.sh r3c5 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --dist --steps 50 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/r3c5/bench_dist_n1.json 2> gpurun_out/r3c5/bench_dist_n1.err && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 1 --dist --publish --steps 50 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/r3c5/bench_dist_n1_publish.json 2> gpurun_out/r3c5/bench_dist_n1_publish.err
