# GLSL kernel change: parity, timing, then per-wave work counters (instrumented rebuild).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-glsl_ab}
mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_glsl.py -q -m gpu -rf -x > $O/glsl_tests.log 2>&1; echo "tests exit $?" >> $O/glsl_tests.log
grep -q " passed" $O/glsl_tests.log || exit 1
grep -q "failed" $O/glsl_tests.log && exit 1
timeout -k 10 300 python tools/bench_glsl.py --no-cpu --variants ${GV:-0} > $O/glsl.json 2>&1 || exit 1
if [ -f tools/instrument_glsl.py ]; then
  python tools/instrument_glsl.py sfml-software-raytracer_amd/csrc/glsl_trace.hip && \
  sed -i 's/-fvisibility=hidden //' sfml-software-raytracer_amd/Makefile && \
  make -C sfml-software-raytracer_amd -j16 > $O/stats_build.log 2>&1 && \
  timeout -k 10 300 python tools/glsl_work_counters.py > $O/stats.txt 2>&1
fi
echo done
