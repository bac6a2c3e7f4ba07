# Round pass on the current tree plus exact block counts of the voxel and GLSL kernels:
#   /usr/local/graft/bin/gpurun --timeout 1800 -- "TAG=r5h bash tools/gpu/r5h.sh"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:?}
mkdir -p gpurun_out/$T
TAG=$T/pass bash tools/gpu/pass.sh || exit 1
for k in voxel glsl; do
  timeout -k 10 180 python tools/isa_block_profile.py run $k > gpurun_out/$T/bbcounts_$k.json 2> gpurun_out/$T/bb_$k.err || exit 1
done
TAG=$T/prof bash tools/gpu/prof_all.sh || exit 1
echo all done
