#!/bin/bash
# All -m gpu tests in one process, bounded; log under gpurun_out/<tag>/tests.log
set -o pipefail
TAG=${1:-tests}
shift
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v -rf --timeout 600 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/$TAG/tests.log | grep -c PASSED
tail -40 gpurun_out/$TAG/tests.log | grep -v "^  " | tail -25
exit $rc
