set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-glsl}
mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_glsl.py -q -m gpu -rf -x > $O/glsl_tests.log 2>&1; echo "tests exit $?" >> $O/glsl_tests.log
grep -q "passed" $O/glsl_tests.log || exit 1
grep -q "failed\|error" $O/glsl_tests.log && exit 1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -k acosf -rf > $O/acosf.log 2>&1 || exit 1
timeout -k 10 600 python tools/bench_glsl.py > $O/bench_glsl.json 2>&1 || exit 1
echo done
