# GLSL A/B of prebuilt libraries (LIBS=a.so,b.so[^O]), the GLSL GPU tests, the block counts of
# the current source (tools/glsl_block_profile.py run) and the GLSL kernel trace + PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-glslab}
mkdir -p $O
P=sfml-software-raytracer_amd
timeout -k 10 400 python -u tools/ab_libs.py --libs ${LIBS:?set LIBS=a.so,b.so} \
  --rounds 3 --reps 60 --cases glsl1080,glsl4k > $O/ab.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_glsl.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/glsl_block_profile.py run > $O/glsl_counts.json 2> $O/glsl_counts.err || exit 1
TAG=$TAG/glsl bash tools/gpu/prof_glsl.sh || exit 1
echo done
