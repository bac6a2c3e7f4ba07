# Selected GPU tests: TAG=<name> SEL="<pytest -k expr>" FILES="<test files>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tests}
mkdir -p $O
timeout -k 10 ${TMO:-900} python -u -m pytest ${FILES:-tests} -m gpu -x -v -rf --timeout 300 --timeout-method thread \
  ${SEL:+-k "$SEL"} --durations=20 > $O/gpu_tests.log 2>&1
rc=$?
echo "tests exit $rc" >> $O/gpu_tests.log
exit $rc
