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
echo done
