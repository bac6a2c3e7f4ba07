# Voxel A/B of prebuilt libraries (LIBS=a.so,b.so[^O]), the voxel and stream GPU tests, then the
# voxel kernel trace + PMC passes (tools/gpu/prof_voxel.sh), under gpurun_out/$TAG/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-vox2}
mkdir -p $O
P=sfml-software-raytracer_amd
timeout -k 10 400 python -u tools/ab_libs.py --libs ${LIBS:?set LIBS=a.so,b.so} \
  --rounds 3 --reps 60 --cases vox1080,vox4k,vox4k_rot > $O/ab.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_voxel.py tests/test_streams.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
TAG=$TAG/voxel bash tools/gpu/prof_voxel.sh || exit 1
echo done
