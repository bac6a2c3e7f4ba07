# Full sphere parity file (incl. the random-scene tests), then the kernel-time probe with
# VARIANTS (march / outside ...) x KV (SFRT_OPT_VARIANT list).  TAG names the output dir.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-iter2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -20 $O/tests.log; exit 1; }
timeout -k 10 300 python tools/perf_probe.py --variants ${VARIANTS:-march,outside} --kvariants ${KV:-0} > $O/probe.txt 2>&1 || exit 1
tail -3 $O/tests.log
grep -v "^{" $O/probe.txt
