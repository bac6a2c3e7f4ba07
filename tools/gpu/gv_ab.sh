# GLSL one-wave-workgroup variant and the voxel 8x8 tile build, timed against the defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-gv_ab}
mkdir -p $O
timeout -k 10 300 python tools/bench_glsl.py --no-cpu --variants 0,2,0,2 > $O/glsl.json 2>&1 || exit 1
timeout -k 10 300 python tools/bench_voxel.py --no-cpu > $O/voxel16.json 2>&1 || exit 1
make -s -C sfml-software-raytracer_amd clean > /dev/null && make -s -C sfml-software-raytracer_amd -j16 EXTRA=-DSFRT_VOXEL_TILE8 > $O/build8.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_voxel.py --no-cpu > $O/voxel8.json 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests/test_voxel.py -q -m gpu -x > $O/voxel8_tests.log 2>&1; tail -2 $O/voxel8_tests.log
echo done
