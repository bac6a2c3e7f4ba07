# Voxel variants A/B (SFRT_VOX_VARIANT builds under sfml-software-raytracer_amd/build_v*/) and the
# GLSL block profile (tools/glsl_block_profile.py run), under gpurun_out/$TAG/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-voxab}
mkdir -p $O
P=sfml-software-raytracer_amd
timeout -k 10 500 python -u tools/ab_libs.py --libs ${LIBS:-$P/libsfrt.so,$P/build_v1/libsfrt.so,$P/build_v2/libsfrt.so,$P/build_v3/libsfrt.so,$P/build_v5/libsfrt.so,$P/build_v7/libsfrt.so} \
  --rounds 3 --reps 60 --cases vox1080,vox4k,vox4k_rot > $O/ab.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/glsl_block_profile.py run > $O/glsl_blocks.json 2> $O/glsl_blocks.err || exit 1
echo done
