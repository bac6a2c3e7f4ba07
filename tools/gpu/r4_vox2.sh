# Voxel: A/B of the round-3 library (build_prev) against the new kernel (and the spilling v5
# build), the voxel GPU tests, then the voxel kernel trace + PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-vox2}
mkdir -p $O
P=sfml-software-raytracer_amd
timeout -k 10 400 python -u tools/ab_libs.py --libs ${LIBS:-$P/build_prev/libsfrt.so,$P/libsfrt.so} \
  --rounds 3 --reps 60 --cases vox1080,vox4k,vox4k_rot > $O/ab.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_voxel.py tests/test_streams.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
TAG=$TAG/voxel bash tools/gpu/prof_voxel.sh || exit 1
echo done
