# One GPU pass: the whole -m gpu suite, smoke(), the default bench line, then a kernel
# trace of the same bench command (the profile the bench line's kernel time must agree with).
#   /usr/local/graft/bin/gpurun --timeout 1200 -- "TAG=r2a bash tools/gpu/pass.sh"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pass}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
  --durations=15 > $O/gpu_tests.log 2>&1
echo "tests exit $?" >> $O/gpu_tests.log
grep -q " passed" $O/gpu_tests.log || exit 1
grep -q "failed\|Fatal\|core dumped\|Timeout" $O/gpu_tests.log && exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python bench.py --steps 100 --warmup 20 --no-cpu-baseline --headline-only > $O/bench_trace.json 2> $O/bench_trace.err || exit 1
echo done
