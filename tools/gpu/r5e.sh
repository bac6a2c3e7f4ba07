# Round-5 check of the voxel/GLSL changes: their GPU tests and the bench rehearsal, block counts
# (tools/isa_block_profile.py) and the kernel traces + PMC passes, under gpurun_out/r5e/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_voxel.py tests/test_glsl.py tests/test_streams.py tests/test_bench_rehearsal.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
for k in voxel glsl; do
  timeout -k 10 180 python tools/isa_block_profile.py run $k > $O/bbcounts_$k.json 2> $O/bb_$k.err || exit 1
done
TAG=r5e/voxel bash tools/gpu/prof_voxel.sh || exit 1
TAG=r5e/glsl bash tools/gpu/prof_glsl.sh || exit 1
echo done
