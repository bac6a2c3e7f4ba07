set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-voxel}
mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_voxel.py -q -m gpu -rf > $O/voxel_tests.log 2>&1; echo "tests exit $?" >> $O/voxel_tests.log
timeout -k 10 600 python tools/bench_voxel.py > $O/bench_voxel.json 2>&1 || exit 1
echo done
