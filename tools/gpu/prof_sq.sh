# Extra SQ counter passes of the headline bench command (issue/stall breakdown):
#   /usr/local/graft/bin/gpurun --timeout 600 -- "TAG=r3i bash tools/gpu/prof_sq.sh"
# summarise with tools/rocprof_summary.py --sq gpurun_out/$TAG/sq_a gpurun_out/$TAG/sq_b ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-prof_sq}
mkdir -p $O
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --headline-only"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_IFETCH SQ_IFETCH_LEVEL SQ_ACTIVE_INST_MISC -d $O/sq_a -o run --output-format csv -- python $B > $O/sq_a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_INST_LEVEL_SMEM SQ_INST_CYCLES_SMEM SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT -d $O/sq_b -o run --output-format csv -- python $B > $O/sq_b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_LEVEL_WAVES SQ_CYCLES -d $O/sq_c -o run --output-format csv -- python $B > $O/sq_c.log 2>&1 || exit 1

# VALU of the march alone (-DSFRT_EXP=64 build: no shading tail) against the release build
if [ -f sfml-software-raytracer_amd/build_x64/libsfrt.so ]; then
  SFRT_LIB=sfml-software-raytracer_amd/build_x64/libsfrt.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VALU_TRANS_F32 -d $O/sq_x64 -o run --output-format csv -- python tools/frame_loop.py 50 > $O/sq_x64.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VALU_TRANS_F32 -d $O/sq_rel -o run --output-format csv -- python tools/frame_loop.py 50 > $O/sq_rel.log 2>&1 || exit 1
fi
echo done all
