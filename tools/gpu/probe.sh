set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${PROBE_TAG:-probe}
mkdir -p $O
timeout -k 10 300 python tools/perf_probe.py > $O/probe.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $O/pmc -o run --output-format csv -- python tools/perf_probe.py --reps 2 --rounds 1 > $O/probe_pmc.txt 2>&1 || exit 1
echo done
