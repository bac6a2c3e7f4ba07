# Kernel-variant A/B for the sphere path: variant parity, then timings.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-kv}
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -rf -k "variants or oracle" > $O/tests.log 2>&1; echo "tests exit $?" >> $O/tests.log
timeout -k 10 600 python tools/perf_probe.py --rounds 3 --variants march --kvariants ${KV:-0} > $O/probe.txt 2>&1 || exit 1
echo done
