set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-voxel_ab}
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -rf -k "div_recip" > $O/div.log 2>&1; echo "exit $?" >> $O/div.log
timeout -k 10 900 python -m pytest tests/test_voxel.py -q -m gpu -rf -x > $O/voxel_tests.log 2>&1; echo "tests exit $?" >> $O/voxel_tests.log
grep -q " passed" $O/voxel_tests.log || exit 1
grep -q "failed" $O/voxel_tests.log && exit 1
timeout -k 10 300 python tools/bench_voxel.py --no-cpu > $O/voxel.json 2>&1 || exit 1
echo done
