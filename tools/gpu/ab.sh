# Build-flag A/B: parity for all three renderers, then kernel timings.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}
mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_glsl.py tests/test_voxel.py -q -m gpu -rf -x > $O/gpu_tests.log 2>&1; echo "tests exit $?" >> $O/gpu_tests.log
timeout -k 10 600 python tools/perf_probe.py --rounds 3 --variants march --kvariants ${KV:-0} > $O/probe.txt 2>&1 || exit 1
timeout -k 10 300 python tools/bench_glsl.py --no-cpu > $O/glsl.json 2>&1 || exit 1
timeout -k 10 300 python tools/bench_voxel.py --no-cpu > $O/voxel.json 2>&1 || exit 1
echo done
