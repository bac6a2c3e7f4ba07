# A/B of prebuilt libraries per renderer (VLIBS voxel, GLIBS GLSL, SLIBS sphere), the GPU tests of
# each candidate (VCAND, GCAND, SCAND) and block counts of instrumented variants (BB="kernel:variant";
# tools/isa_block_profile.py), under gpurun_out/$TAG/:
#   VLIBS=a.so,b.so VCAND=b.so GLIBS=a.so,c.so GCAND=c.so BB="voxel:base glsl:gl" TAG=r6x bash tools/gpu/ab_kernels.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:?}
mkdir -p $O
if [ -n "$VLIBS" ]; then
  timeout -k 10 400 python -u tools/ab_libs.py --libs $VLIBS --rounds ${ROUNDS:-3} --reps 60 \
    --cases ${VCASES:-vox1080,vox4k,vox4k_rot} > $O/ab_voxel.txt 2>&1 || exit 1
fi
if [ -n "$GLIBS" ]; then
  timeout -k 10 400 python -u tools/ab_libs.py --libs $GLIBS --rounds ${ROUNDS:-3} --reps 40 \
    --cases ${GCASES:-glsl1080,glsl4k,glsl4k_move} > $O/ab_glsl.txt 2>&1 || exit 1
fi
if [ -n "$SLIBS" ]; then
  timeout -k 10 400 python -u tools/ab_libs.py --libs $SLIBS --rounds ${ROUNDS:-3} --reps 60 \
    --cases ${SCASES:-4k,4k_rot,4k_turn,1080} > $O/ab_sphere.txt 2>&1 || exit 1
fi
if [ -n "$VCAND" ]; then
  SFRT_LIB=$VCAND timeout -k 10 400 python -u -m pytest tests/test_voxel.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_voxel.log 2>&1 || exit 1
fi
if [ -n "$GCAND" ]; then
  SFRT_LIB=$GCAND timeout -k 10 400 python -u -m pytest tests/test_glsl.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_glsl.log 2>&1 || exit 1
fi
if [ -n "$SCAND" ]; then
  SFRT_LIB=$SCAND timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_sphere.log 2>&1 || exit 1
fi
for kv in $BB; do
  k=${kv%%:*}; v=${kv#*:}
  if [ "$v" = "$k" ] || [ "$v" = base ]; then
    timeout -k 10 180 python tools/isa_block_profile.py run $k > $O/bbcounts_${k}.json 2> $O/bb_${k}.err || exit 1
  else
    timeout -k 10 180 python tools/isa_block_profile.py run $k --variant $v > $O/bbcounts_${k}_$v.json 2> $O/bb_${k}_$v.err || exit 1
  fi
done
echo done
