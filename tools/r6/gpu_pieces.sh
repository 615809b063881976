#!/bin/bash
# Round 6: the multi-piece sharded window + every partition / exchange test.
set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 1000 python -u -m pytest -x -v --durations=0 --timeout 400 --timeout-method thread \
    tests/test_gpu_local_world.py tests/test_gpu_multi.py \
    "tests/test_gpu_round4.py::test_partition_runs_voxelize_runs_match_oracle" \
    > gpurun_out/r6b/pytest_pieces.log 2>&1
rc=$?
tail -60 gpurun_out/r6b/pytest_pieces.log
exit $rc
