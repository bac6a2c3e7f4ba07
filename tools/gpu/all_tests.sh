# Whole GPU suite, then the default bench line and smoke().
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-all}
mkdir -p $O
timeout -k 10 1200 python -m pytest tests -q -m gpu -rf --durations=10 > $O/gpu_tests.log 2>&1; echo "tests exit $?" >> $O/gpu_tests.log
grep -q " passed" $O/gpu_tests.log || exit 1
grep -q "Fatal\|core dumped" $O/gpu_tests.log && exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
echo done
