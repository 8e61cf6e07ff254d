set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/${TAG:-r07b}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- python3 $ROOT/bench.py --mode ${MODE:-B} --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-roofline > $OUT/tr.log 2>&1 || { tail -20 $OUT/tr.log; exit 1; }
cd $ROOT
T=$(find $OUT -name '*kernel_trace.csv' | head -1)
python3 tools/copy_census.py $T --match CUDAFunctor_add > $OUT/adds.txt 2>&1
gzip $T
tail -3 $OUT/adds.txt
