# Kernel trace + PMC passes of tools/bench_voxel.py (profiles/<tag>_voxel_*):
#   /usr/local/graft/bin/gpurun --timeout 900 -- "TAG=r2m bash tools/gpu/prof_voxel.sh"
# then: python tools/rocprof_summary.py --kernel k_voxel --trace gpurun_out/$TAG/trace
#       --fetch gpurun_out/$TAG/pmc_fetch --write gpurun_out/$TAG/pmc_write
#       --sq gpurun_out/$TAG/pmc_sq gpurun_out/$TAG/pmc_sq2 --tag ${TAG}_voxel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-profvox}
mkdir -p $O
B="tools/bench_voxel.py --no-cpu --steps 20 --set bench"
# the kernel trace over 300 frames per launch size (20 frames sit in the clock ramp: their
# average runs 3-7 % above the bench line's); the PMC passes keep 20
BT="tools/bench_voxel.py --no-cpu --steps 300 --set bench"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python $BT > $O/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python $B > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python $B > $O/pmc_write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_sq -o run --output-format csv -- python $B > $O/pmc_sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $O/pmc_sq2 -o run --output-format csv -- python $B > $O/pmc_sq2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $O/pmc_sq3 -o run --output-format csv -- python $B > $O/pmc_sq3.log 2>&1 || exit 1
echo done
