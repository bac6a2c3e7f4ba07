# Interleaved A/B of prebuilt libraries (tools/ab_libs.py), then optionally selected GPU tests:
#   /usr/local/graft/bin/gpurun --timeout 900 -- "TAG=r3c LIBS=a.so,b.so CASES=4k,8k SEL='parity' bash tools/gpu/ab.sh"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}
mkdir -p $O
timeout -k 10 ${ABTMO:-600} python -u tools/ab_libs.py --libs "$LIBS" --rounds ${ROUNDS:-3} --reps ${REPS:-60} \
  --cases ${CASES:-4k,4k_rot,4k_turn,8k,1080,4k_256} > $O/ab.txt 2>&1 || exit 1
if [ -n "$SEL$FILES" ]; then
  timeout -k 10 ${TMO:-600} python -u -m pytest ${FILES:-tests} -m gpu -x -q -rf --timeout 300 --timeout-method thread \
    ${SEL:+-k "$SEL"} > $O/gpu_tests.log 2>&1
  rc=$?
  echo "tests exit $rc" >> $O/gpu_tests.log
  exit $rc
fi
echo done
