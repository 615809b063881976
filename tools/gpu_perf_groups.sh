# bench (driver settings) + kernel traces of the 4K single-frame and C3 workloads, and of 4K frames
# one at a time (tools/frame_driver.py: per-kernel durations without frames in flight overlapping)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-perf}; mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/t4k -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --width 3840 --height 2160 --batch 1 --no-secondary --no-cpu-baseline --no-kernel-timing > $O/t4k.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/tc3 -o run --output-format csv -- python3 tools/bench_c3.py --steps 5 > $O/tc3.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/s4k -o run --output-format csv -- python3 tools/frame_driver.py 3840 2160 4 0 20 dense > $O/s4k.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/sc2 -o run --output-format csv -- python3 tools/frame_driver.py 640 480 4 0 100 dense 8 > $O/sc2.log 2>&1 || exit 1
