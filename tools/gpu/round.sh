# One GPU pass for a tag: the -m gpu suite, smoke(), the default bench line, the kernel trace
# of the bench command and the PMC passes, all under gpurun_out/<tag>/.  PROF=all profiles the
# voxel and GLSL kernels too (tools/gpu/prof_all.sh, else tools/gpu/prof.sh: the headline only);
# BB="voxel glsl ..." adds exact block counts of those kernels (tools/isa_block_profile.py).
#   /usr/local/graft/bin/gpurun --timeout 1500 -- "PROF=all BB='voxel glsl' bash tools/gpu/round.sh <tag>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-round}
TAG=$T/pass bash tools/gpu/pass.sh || exit 1
mkdir -p gpurun_out/$T
for k in $BB; do
  timeout -k 10 180 python tools/isa_block_profile.py run $k > gpurun_out/$T/bbcounts_$k.json 2> gpurun_out/$T/bb_$k.err || exit 1
done
if [ "$PROF" = all ]; then
  TAG=$T/prof bash tools/gpu/prof_all.sh || exit 1
else
  TAG=$T/prof bash tools/gpu/prof.sh || exit 1
fi
echo round done
