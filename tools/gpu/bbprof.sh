# Block execution counts of the instrumented kernels (tools/isa_block_profile.py, built here
# beforehand with `python tools/isa_block_profile.py build KERNEL`), under gpurun_out/$TAG/:
#   /usr/local/graft/bin/gpurun --timeout 600 -- "TAG=r5b KERNELS='voxel sphere glsl' bash tools/gpu/bbprof.sh"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:?}
mkdir -p $O
for k in ${KERNELS:-voxel sphere glsl}; do
  timeout -k 10 180 python tools/isa_block_profile.py run $k > $O/bbcounts_$k.json 2> $O/bbcounts_$k.err || exit 1
done
echo done
