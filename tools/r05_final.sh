#!/bin/bash
# Round-5 closing evidence: the -m gpu suite, smoke(), the default bench line, mode-A kernel stats + PMC.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r05f2}
timeout -k 10 900 python -u -m pytest -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread tests > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 800 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-300 gpurun_out/${TAG}_bench.json
exit $rc
