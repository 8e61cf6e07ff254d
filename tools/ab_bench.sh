#!/bin/bash
# Interleaved A/B of library variants ab/<name>.so on the bench's encoder-forward
# north star and step throughput: usage: bash tools/ab_bench.sh ROUNDS name1 name2 ...
set -o pipefail
R=${1:?rounds}; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for n in "$@"; do
    DMF_HIP_LIB=ab/$n.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --steps 30 --warmup 5 $AB_ARGS > gpurun_out/ab/$n.$r.json 2> gpurun_out/ab/$n.$r.err || { echo "bench $n failed"; tail -20 gpurun_out/ab/$n.$r.err; exit 1; }
    python - "$n" "$r" <<'PY'
import json, sys
n, r = sys.argv[1], sys.argv[2]
d = json.loads(open(f"gpurun_out/ab/{n}.{r}.json").read().strip().splitlines()[-1])
print(f"{n:10s} round {r}: {d['value']:8.1f} vol/s  {d['ms_per_step']:7.3f} ms/step  enc fwd {d.get('encoder_forward', {}).get('ms', float('nan')):6.3f} ms", flush=True)
PY
  done
done
