bash tools/gpu_tests.sh r02f; rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash tools/prof_enc.sh r02f_prof
