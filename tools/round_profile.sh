#!/bin/bash
# Everything a round's profiles/ needs, in one GPU call:
# GPU tests, bench (with the per-launch conv dump), rocprofv3 kernel stats,
# and the two PMC passes for HBM traffic. usage: gpurun -- bash tools/round_profile.sh TAG
set -o pipefail
TAG=${1:?tag}
bash tools/gpu_session.sh $TAG all || exit 1
bash tools/pmc_session.sh ${TAG}_pmc || exit 1
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc --json gpurun_out/$TAG/pmc_traffic.json
