set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${PROBE_TAG:-slots}
mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -rf -x > $O/gpu_tests.log 2>&1; echo "tests exit $?" >> $O/gpu_tests.log
for S in 0 4 6 8; do SFRT_SLOTS=$S timeout -k 10 300 python tools/perf_probe.py --rounds 2 > $O/probe_s$S.txt 2>&1 || exit 1; done
for S in 0 8; do SFRT_SLOTS=$S timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $O/pmc_s$S -o run --output-format csv -- python tools/perf_probe.py --reps 2 --rounds 1 > $O/pmc_s$S.txt 2>&1 || exit 1; done
echo done
