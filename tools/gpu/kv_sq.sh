# SQ instruction/stall counters per sphere-kernel variant (perf_probe drives the variants).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-kvsq}
mkdir -p $O
P="tools/perf_probe.py --rounds 1 --reps 5 --variants march --kvariants ${KV:-0}"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES -d $O/a -o run --output-format csv -- python3 $P > $O/a.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES -d $O/b -o run --output-format csv -- python3 $P > $O/b.log 2>&1 || exit 1
echo done
