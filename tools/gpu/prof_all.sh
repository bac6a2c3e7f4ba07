# Kernel trace + PMC passes of all three kernels (voxel, GLSL, headline sphere) under gpurun_out/$TAG/{voxel,glsl,sphere}
#   /usr/local/graft/bin/gpurun --timeout 1500 -- "TAG=r5a bash tools/gpu/prof_all.sh"
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:?}/voxel bash tools/gpu/prof_voxel.sh || exit 1
TAG=${TAG:?}/glsl bash tools/gpu/prof_glsl.sh || exit 1
TAG=${TAG:?}/sphere bash tools/gpu/prof.sh || exit 1
echo all done
