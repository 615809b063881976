#!/bin/bash
# Round 6: the local-world step tests under the strict transport + the facade component.
set -o pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_local_world.py tests/test_facade_gpu.py > gpurun_out/r6a/pytest_local.log 2>&1
rc=$?
tail -30 gpurun_out/r6a/pytest_local.log
exit $rc
