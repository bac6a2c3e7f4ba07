set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-display}
mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -rf -x > $O/gpu_tests.log 2>&1; echo "tests exit $?" >> $O/gpu_tests.log
timeout -k 10 600 python tools/bench_display.py > $O/display.json 2>&1 || exit 1
echo done
