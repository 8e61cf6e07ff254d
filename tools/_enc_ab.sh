# encoder forward with the persistent conv on / off (same process order alternated)
set -o pipefail
for v in 1 0 1 0; do
  DMF_PS=$v timeout -k 10 200 python tools/enc_fwd_prof.py --reps 20 2>/dev/null | sed "s/^/ps=$v /" || exit 1
done
DMF_PS=1 timeout -k 10 200 python tools/enc_fwd_prof.py --reps 20 --serial 2>/dev/null | sed "s/^/ps=1 /" || exit 1
DMF_PS=0 timeout -k 10 200 python tools/enc_fwd_prof.py --reps 20 --serial 2>/dev/null | sed "s/^/ps=0 /" || exit 1
