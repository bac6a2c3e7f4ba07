# Voxel A/B of prebuilt libraries + the GPU voxel tests on a candidate + block counts of
# instrumented variants, under gpurun_out/$TAG/:
#   LIBS=a.so,b.so CAND=b.so BBVARIANTS="ul:SFRT_VOX_ULOOP=1" TAG=r5c bash tools/gpu/ab_vox_r5.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:?}
mkdir -p $O
timeout -k 10 400 python -u tools/ab_libs.py --libs ${LIBS:?} --rounds ${ROUNDS:-3} --reps 60 \
  --cases ${CASES:-vox1080,vox4k,vox4k_rot} > $O/ab.txt 2>&1 || exit 1
if [ -n "$CAND" ]; then
  SFRT_LIB=$CAND timeout -k 10 400 python -u -m pytest tests/test_voxel.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
fi
for v in ${BBVARIANTS}; do
  tag=${v%%:*}
  if [ "$tag" = base ]; then
    timeout -k 10 180 python tools/isa_block_profile.py run ${BBKERNEL:-voxel} > $O/bbcounts_base.json 2> $O/bb_base.err || exit 1
  else
    timeout -k 10 180 python tools/isa_block_profile.py run ${BBKERNEL:-voxel} --variant $tag > $O/bbcounts_$tag.json 2> $O/bb_$tag.err || exit 1
  fi
done
echo done
