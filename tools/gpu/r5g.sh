# GLSL wall cull: A/B against the previous build, the GLSL GPU tests, block counts, PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:?}
mkdir -p $O
A=sfml-software-raytracer_amd/build_ab
timeout -k 10 600 python -u -m pytest tests/test_glsl.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/ab_libs.py --libs $A/lib_head.so,$A/lib_wc.so --rounds 3 --reps 40 \
  --cases glsl1080,glsl4k,glsl4k_move,glsl1080_move > $O/ab_glsl.txt 2>&1 || exit 1
timeout -k 10 180 python tools/isa_block_profile.py run glsl > $O/bbcounts_glsl.json 2> $O/bb_glsl.err || exit 1
TAG=${TAG}/glsl bash tools/gpu/prof_glsl.sh || exit 1
if [ -n "$VOX" ]; then
  timeout -k 10 400 python -u tools/ab_libs.py --libs $A/lib_wc.so,$A/lib_mk.so,$A/lib_mki.so,$A/lib_mkic.so,$A/lib_mall.so --rounds 3 --reps 60 \
    --cases vox1080,vox4k,vox4k_rot > $O/ab_voxel.txt 2>&1 || exit 1
  SFRT_LIB=$A/lib_mall.so timeout -k 10 400 python -u -m pytest tests/test_voxel.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_voxel.log 2>&1 || exit 1
fi
echo done
