set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_voxel.py tests/test_glsl.py tests/test_streams.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
for k in voxel glsl; do
  timeout -k 10 180 python tools/isa_block_profile.py run $k > $O/bbcounts_$k.json 2> $O/bb_$k.err || exit 1
done
TAG=r5e/voxel bash tools/gpu/prof_voxel.sh || exit 1
TAG=r5e/glsl bash tools/gpu/prof_glsl.sh || exit 1
echo done
