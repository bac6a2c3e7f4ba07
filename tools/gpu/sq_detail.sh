# Extra SQ counters (branch/ifetch/divergence/transcendentals) for the sphere kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-sqd}
mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_IFETCH SQ_IFETCH_LEVEL SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VSKIPPED SQ_INST_CYCLES_SALU -d $O/sqd -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > $O/sqd.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_VALU -d $O/sqe -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extra > $O/sqe.log 2>&1 || exit 1
echo done
