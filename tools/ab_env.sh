#!/bin/bash
# Interleaved A/B of knob settings (dmf_ops.KNOBS, passed as bench.py --knob) on the bench's
# encoder-forward north star and step throughput (same library):
#   bash tools/ab_env.sh ROUNDS "wgrad_sq=0" "wgrad_sq=1" ...   (a setting may hold several: "a=1,b=0"; "-" = defaults)
#   AB_ARGS="--mode B" bash tools/ab_env.sh ...                  (extra bench.py arguments for every run)
set -o pipefail
R=${1:?rounds}; shift
mkdir -p gpurun_out/abenv
for r in $(seq 1 $R); do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    K=""
    if [ "$e" != "-" ]; then for kv in ${e//,/ }; do K="$K --knob $kv"; done; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 30 --warmup 5 $AB_ARGS $K > gpurun_out/abenv/$i.$r.json 2> gpurun_out/abenv/$i.$r.err || { echo "bench $e failed"; tail -20 gpurun_out/abenv/$i.$r.err; exit 1; }
    python - "$e" gpurun_out/abenv/$i.$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:28s} {d['value']:8.1f} vol/s  {d['ms_per_step']:7.3f} ms/step  enc fwd {d.get('encoder_forward', {}).get('ms', float('nan')):6.3f} ms", flush=True)
PY
  done
done
